set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${TAG:-ab}; mkdir -p $O
export TMPDIR=/tmp
for v in default a b c; do
  if [ $v = default ]; then L=""; else L=$PWD/tools/forensic/_ref/libheist_ab_$v.so; fi
  for rep in 1 2; do
    HEIST_LIB=$L PROBE_STAMPS=1 timeout -k 10 120 python tools/probe_policy.py 2>/dev/null | grep phase > $O/stamps_${v}_$rep.log || exit 1
    HEIST_LIB=$L PROBE_N=4096 timeout -k 10 120 python tools/probe_policy.py 2>/dev/null | grep backbone > $O/probe_${v}_$rep.log || exit 1
    echo "$v $rep $(python3 -c "import json;d=json.load(open('$O/stamps_${v}_$rep.log'));print(d['env_cycles_median'], d['phase_median_cycles']['conv2_mfma'], d['phase_median_cycles']['conv3'])") $(python3 -c "import json;d=json.load(open('$O/probe_${v}_$rep.log'));print(d['backbone_kernel_ms'], d['mfma_frac_of_2500'])")"
  done
done

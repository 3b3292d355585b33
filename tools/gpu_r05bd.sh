#!/bin/bash
# conv2 pass boundaries (HEIST_CONV2_SASB) 3,6 / 2,5 / 4,6 vs the product (3,5);
# settled backbone timing (bench.measure_policy) and phase stamps.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05bd}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep '^{' $OUT/$name.log | cut -c1-260; if fatal $rc; then exit $rc; fi; }
for i in 1 2; do
  for v in prod s36 s25 s46; do
    L=""; [ $v != prod ] && L=$PWD/tools/bin/libheist_hip_$v.so
    HEIST_LIB=$L run bb_${v}_$i 120 python3 -c "import json,torch,bench; d=torch.device('cuda:0'); [print(json.dumps({'n':n,'ms':bench.measure_policy(d,n)['backbone_roofline']['kernel_ms'],'frac':bench.measure_policy(d,n)['backbone_roofline']['frac']}),flush=True) for n in (4096,16384)]"
    HEIST_LIB=$L PROBE_STAMPS=1 run st_${v}_$i 120 python3 tools/probe_policy.py
  done
done
echo "== all done"

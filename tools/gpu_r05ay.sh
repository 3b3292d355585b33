#!/bin/bash
# conv3 split-tile A/B: policy parity tests, then the backbone timing (bench.measure_policy)
# and phase stamps, product build vs the previous heist_policy.hip (tools/bin/libheist_hip_polbase.so).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05ay}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 $OUT/$name.log | cut -c1-200; if fatal $rc; then exit $rc; fi; }
run pytest_policy 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_policy.py
for i in 1 2; do
  for v in prod polbase; do
    L=""; [ $v != prod ] && L=$PWD/tools/bin/libheist_hip_$v.so
    HEIST_LIB=$L run bb_${v}_$i 120 python3 -c "import json,torch,bench; d=torch.device('cuda:0'); [print(json.dumps({'n':n,'bb':bench.measure_policy(d,n)['backbone_roofline']}),flush=True) for n in (4096,16384)]"
    HEIST_LIB=$L PROBE_STAMPS=1 run st_${v}_$i 120 python3 tools/probe_policy.py
  done
done
echo "== all done"

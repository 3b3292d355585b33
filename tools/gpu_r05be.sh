#!/bin/bash
# Backbone prologue (conv2 fragment copy unrolled, first observation load hoisted): policy
# parity tests on the variant, then settled backbone timing, variant vs product, twice.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05be}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep '^{' $OUT/$name.log | cut -c1-200; tail -n 1 $OUT/$name.log | cut -c1-120; if fatal $rc; then exit $rc; fi; }
HEIST_LIB=$PWD/tools/bin/libheist_hip_pro.so run pytest_policy 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_policy.py tests/test_gpu_train_backbone.py
for i in 1 2; do
  for v in prod pro; do
    L=""; [ $v != prod ] && L=$PWD/tools/bin/libheist_hip_$v.so
    HEIST_LIB=$L run bb_${v}_$i 120 python3 -c "import json,torch,bench; d=torch.device('cuda:0'); [print(json.dumps({'n':n,'ms':r['backbone_roofline']['kernel_ms'],'frac':r['backbone_roofline']['frac']}),flush=True) for n in (1024,4096,16384) for r in [bench.measure_policy(d,n)]]"
  done
done
echo "== all done"

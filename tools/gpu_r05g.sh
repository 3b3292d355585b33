#!/bin/bash
# Fused fp32 training tail: parity tests, then the training iteration A/B (HEIST_FUSED_TRAIN)
# and its kernel breakdown.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05g}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
run pytest_train 600 python -u -m pytest tests/test_gpu_train_backbone.py tests/test_gpu_policy.py tests/test_gpu_trainer.py -x -v --timeout 300 --timeout-method thread
run train_fused 600 python3 tools/probe_train.py
HEIST_FUSED_TRAIN=0 run train_plain 600 python3 tools/probe_train.py
run prof_train 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_train -o train --output-format csv -- python3 tools/probe_train.py
echo "== all done"

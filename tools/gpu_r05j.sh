#!/bin/bash
# Lean-kernel phase stamps (architect + synthetic layouts) and the lean/multi env tests
# (STAMP=false instances must be unchanged).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05j}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 $OUT/$name.log | cut -c1-300; if fatal $rc; then exit $rc; fi; }
run stamps_arch 300 python3 tools/probe_multi_stamps.py
PROBE_LAYOUTS=synthetic run stamps_syn 300 python3 tools/probe_multi_stamps.py
run pytest_lean 900 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 300 --timeout-method thread -k "multi or lean or stamp"
echo "== all done"

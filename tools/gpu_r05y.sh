#!/bin/bash
# Lean kernel with early channel-0/2 stores: env tests, then timings and configs.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05y}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 $OUT/$name.log | cut -c1-160; if fatal $rc; then exit $rc; fi; }
run pytest_env 900 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 300 --timeout-method thread
for i in 1 2; do
  for L in architect synthetic; do
    PROBE_LAYOUTS=$L run ${L}_$i 300 python3 tools/probe_lean_modes.py
  done
  run configs_$i 600 python3 tools/probe_env_configs.py
done
echo "== all done"

#!/bin/bash
# Dispatch order A/B (1: heaviest first, 2: snake draft over the SIMDs) on the env configs
# and the headline; env parity suite under order 2.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05e}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
B="bench.py --no-cpu-baseline --no-secondary --extra-windows 4"
for i in 1 2; do for o in 1 2; do
  HEIST_DISPATCH_ORDER=$o run configs_o${o}_$i 600 python3 tools/probe_env_configs.py
  HEIST_DISPATCH_ORDER=$o run bench_arch_o${o}_$i 300 python3 $B --steps 300 --warmup 30
done; done
HEIST_DISPATCH_ORDER=2 run pytest_env_o2 900 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 300 --timeout-method thread -k "multi or lean"
echo "== all done"

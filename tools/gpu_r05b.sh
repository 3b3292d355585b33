#!/bin/bash
# Interval fans in step_lean_kernel: parity tests, then the synthetic / Architect benches
# (interval fans vs the shared fan table on the Architect layouts).  Architect kernel status tests.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05b}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
B="bench.py --no-cpu-baseline --no-secondary --extra-windows 2"
run pytest_ivl 600 python -u -m pytest tests/test_gpu_env.py -x -v --timeout 300 --timeout-method thread -k "interval_fans or one_wave_per_env or lean_wide or shared_fan"
run bench_syn 300 python3 $B --layouts synthetic --steps 300 --warmup 30
run bench_arch 300 python3 $B --steps 300 --warmup 30
HEIST_SHARED_FAN=0 run bench_arch_ivl 300 python3 $B --steps 300 --warmup 30
run pytest_arch 600 python -u -m pytest tests/test_architect_update.py -x -v --timeout 300 --timeout-method thread -k "timeout or status or graph_path"
echo "== all done"

#!/bin/bash
# One GPU session: the GPU parity suite (or a -k selection), smoke, and the driver's bench
# command line; every step under its own time limit, stopping at the first fatal exit.
# TAG names the output directory gpurun_out/$TAG; PYTEST_K selects tests (default: all -m gpu).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r04x}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
if [ -n "$PYTEST_K" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$PYTEST_K"
elif [ -z "$NO_PYTEST" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
fi
[ -z "$NO_SMOKE" ] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ -n "$PROBE" ] && run probe 300 python3 $PROBE
[ -z "$NO_BENCH" ] && run bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
[ -n "$BENCH_QUICK" ] && run bench_quick 600 python3 bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary
echo "== all done"

#!/bin/bash
# Full GPU suite + smoke, then the training iteration's kernel breakdown (rocprofv3 kernel
# stats of tools/probe_train.py) to see what the Solver's PPO update spends its time on.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05f}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
[ -z "$NO_PYTEST" ] && run pytest_gpu 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
[ -z "$NO_PYTEST" ] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run configs 600 python3 tools/probe_env_configs.py
run bench_arch 300 python3 bench.py --no-cpu-baseline --no-secondary --steps 300 --warmup 30
run prof_train 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_train -o train --output-format csv -- python3 tools/probe_train.py
echo "== all done"

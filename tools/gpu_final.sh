#!/bin/bash
# Final GPU session of a round: GPU parity suite, smoke, default bench, rocprof kernel stats,
# PMC traffic passes, per-probe-mode SQ instruction mix, phase stamps.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r01z}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o heist --output-format csv -- python3 bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o heist --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o heist --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary
run sstamp 300 python tools/probe_step_stamps.py
run pmc_modes 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $OUT/pmc_modes -o modes --output-format csv -- python3 tools/probe_step_modes.py
python tools/pmc_modes.py $OUT/pmc_modes/modes_counter_collection.csv $OUT/pmc_modes.json > /dev/null
run bench 900 python bench.py
# the driver's own command line, last (BENCH_rNN.json runs exactly this)
run bench_driver 900 python3 bench.py --gpus 1 --steps 20 --warmup 5
echo "== all done"

#!/bin/bash
# GPU session: the parity suite, smoke, rocprofv3 kernel stats of the headline bench, PMC
# traffic passes (FETCH_SIZE, WRITE_SIZE), one SQ instruction-mix pass, the driver's bench.
# Each step under its own time limit; the script stops at the first fatal exit.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r04x}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
B="bench.py --no-cpu-baseline --no-secondary"
[ -z "$NO_PYTEST" ] && run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
[ -z "$NO_SMOKE" ] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o heist --output-format csv -- python3 $B --steps 300 --warmup 30
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o heist --output-format csv -- python3 $B --steps 100 --warmup 10
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o heist --output-format csv -- python3 $B --steps 100 --warmup 10
run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $OUT/pmc_sq -o heist --output-format csv -- python3 $B --steps 100 --warmup 10
python tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write --ticks 20 --profile ${TAG:-r04x} --out $OUT/traffic.json > /dev/null
python tools/pmc_sq.py $OUT/pmc_sq --ticks 20 --out $OUT/pmc_sq.json > /dev/null
run bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
echo "== all done"

#!/bin/bash
# Packed interval fans: parity (env suite), then env configs and the synthetic SQ counters.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05d}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
B="bench.py --no-cpu-baseline --no-secondary --extra-windows 2"
run pytest_env 900 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 300 --timeout-method thread
run configs 600 python3 tools/probe_env_configs.py
run bench_arch 300 python3 $B --steps 300 --warmup 30
HEIST_SHARED_FAN=0 run bench_arch_ivl 300 python3 $B --steps 300 --warmup 30
run pmc_sq_syn 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $OUT/pmc_sq_syn -o heist --output-format csv -- python3 $B --layouts synthetic --steps 100 --warmup 10 --extra-windows 0
python tools/pmc_sq.py $OUT/pmc_sq_syn --ticks 20 --out $OUT/pmc_sq_syn.json > /dev/null
echo "== all done"

#!/bin/bash
# Round-5 baseline of the generic K-tick body on the synthetic mix: phase stamps, kernel
# stats and SQ counters of bench.py --layouts synthetic.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05a}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
B="bench.py --no-cpu-baseline --no-secondary --layouts synthetic"
PROBE_LAYOUTS=synthetic run stamps_syn 300 python3 tools/probe_multi_stamps.py
run stamps_arch 300 python3 tools/probe_multi_stamps.py
run bench_syn 300 python3 $B --steps 300 --warmup 30
run prof_syn 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_syn -o heist --output-format csv -- python3 $B --steps 300 --warmup 30
run pmc_sq_syn 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $OUT/pmc_sq_syn -o heist --output-format csv -- python3 $B --steps 100 --warmup 10
python tools/pmc_sq.py $OUT/pmc_sq_syn --ticks 20 --out $OUT/pmc_sq_syn.json > /dev/null
echo "== all done"

#!/bin/bash
# SQ counters of the current step_lean_kernel (synthetic and the headline): three passes each.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05o}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-150; if fatal $rc; then exit $rc; fi; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
P2="SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC"
P3="SQ_WAVES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_BRANCH"
B="bench.py --no-cpu-baseline --no-secondary --steps 60 --warmup 10 --extra-windows 0"
for L in synthetic architect; do
  i=1
  for P in "$P1" "$P2" "$P3"; do
    run pmc_${L}_$i 180 rocprofv3 --pmc $P -d $OUT/pmc_${L}_$i -o heist --output-format csv -- python3 $B --layouts $L
    i=$((i+1))
  done
done
echo "== all done"

#!/bin/bash
# One GPU-box session: build check, GPU parity tests, smoke, bench, rocprof kernel trace.
# Each GPU step has its own time limit; a fault-like exit (abort, segfault, timeout)
# ends the script immediately -- no GPU work after a fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL exit in $name; stopping"; exit $rc; fi
  return 0
}
rocm-smi --showproductname > "$OUT/gpu.txt" 2>&1 || true
nproc > "$OUT/nproc.txt"; lscpu > "$OUT/lscpu.txt" 2>&1
for s in ${STEPS:-pytest smoke bench prof}; do
  case $s in
    pytest) step pytest_gpu 900 python -m pytest tests -m gpu -x -q ;;
    pytestall) step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread ;;
    pytestw) for w in 1 4; do HEIST_STEP_WAVES=$w step pytest_env_w$w 900 python -m pytest tests/test_gpu_env.py -x -q; done ;;
    pytestu) for o in 8; do HEIST_STEP_OCC=$o step pytest_env_o$o 900 python -m pytest tests/test_gpu_env.py -x -q; done ;;
    pytesto8) for w in 1 2 4; do HEIST_STEP_OCC=8 HEIST_STEP_WAVES=$w step pytest_env_w${w}_o8 900 python -m pytest tests/test_gpu_env.py -x -q; done ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    driver) step bench_driver 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    multitest) step pytest_multi 300 python -u -m pytest tests/test_gpu_env.py -k multi -x -v --timeout 200 --timeout-method thread ;;
    quickk) step bench_quick_k 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary ;;
    quickw1) HEIST_MULTI_WAVES=1 step bench_quick_w1 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary ;;
    mstampw1) HEIST_MULTI_WAVES=1 step multi_stamps_w1 300 python tools/probe_multi_stamps.py ;;
    quick1) step bench_quick_1 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary --ticks-per-launch 1 ;;
    quicklicm) HEIST_LIB=$PWD/rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd/heist_amd/libheist_hip_licm.so step bench_quick_licm 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary --ticks-per-launch 1 ;;
    mstamp) step multi_stamps 300 python tools/probe_multi_stamps.py ;;
    profm) step prof_multi 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o heist --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary
           cp "$OUT"/prof/*kernel_stats.csv "$OUT/kernel_stats.csv" 2>/dev/null; true ;;
    pmcm) step pmc_fetch_m 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_m" -o heist --output-format csv -- python3 bench.py --steps 60 --warmup 20 --no-cpu-baseline --no-secondary
          step pmc_write_m 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_m" -o heist --output-format csv -- python3 bench.py --steps 60 --warmup 20 --no-cpu-baseline --no-secondary
          python tools/pmc_traffic.py "$OUT/pmc_fetch_m" "$OUT/pmc_write_m" --ticks 20 --profile ${TAG:-run} --out "$OUT/heist_step_multi_traffic.json" > "$OUT/traffic_m.log" 2>&1; true ;;
    sqm) step pmc_sq_m 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d "$OUT/pmc_sq_m" -o heist --output-format csv -- python3 bench.py --steps 60 --warmup 20 --no-cpu-baseline --no-secondary
         step pmc_sq2_m 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d "$OUT/pmc_sq2_m" -o heist --output-format csv -- python3 bench.py --steps 60 --warmup 20 --no-cpu-baseline --no-secondary
         python tools/pmc_summary.py "$(find "$OUT/pmc_sq_m" -name "*counter_collection.csv" | head -n 1)" step_multi_kernel "$OUT/pmc_sq_m.json" > /dev/null 2>&1
         python tools/pmc_summary.py "$(find "$OUT/pmc_sq2_m" -name "*counter_collection.csv" | head -n 1)" step_multi_kernel "$OUT/pmc_sq2_m.json" > /dev/null 2>&1; true ;;
    archtest) step pytest_arch 600 python -u -m pytest tests/test_architect_update.py tests/test_gpu_trainer.py -k "architect or per_layout or c3" -x -v --timeout 500 --timeout-method thread ;;
    trainq) step bench_train 900 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    agraph) step probe_arch_graph 300 python tools/probe_arch_graph.py ;;
    occ) for o in 8 7 6; do HEIST_MULTI_OCC=$o step bench_occ$o 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary; done
         HEIST_MULTI_OCC=8 step bench_occ8b 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary ;;
    occ1) HEIST_MULTI_OCC=8 step bench_w2o8 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary
          for o in 4 6; do HEIST_MULTI_WAVES=1 HEIST_MULTI_OCC=$o step bench_w1o$o 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary; done
          HEIST_MULTI_OCC=8 step bench_w2o8b 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary ;;
    pab) NP=$PWD/rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd/heist_amd/libheist_hip_nopack.so
         for i in 1 2; do for w in 1 2; do
           HEIST_MULTI_WAVES=$w step bench_pack_w${w}_$i 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary
           HEIST_LIB=$NP HEIST_MULTI_WAVES=$w step bench_nopack_w${w}_$i 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary
         done; done
         for w in 1 2; do HEIST_MULTI_WAVES=$w step bench_syn_w$w 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary --layouts synthetic; done ;;
    drv20) step bench_drv20 300 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline
           step bench_drv20w 300 python bench.py --steps 20 --warmup 20 --no-secondary --no-cpu-baseline
           step bench_drv20k1 300 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --ticks-per-launch 1 ;;
    fanab) for i in 1 2; do for f in 1 0; do
             HEIST_SHARED_FAN=$f step bench_fan${f}_$i 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary
           done; done
           for f in 1 0; do HEIST_SHARED_FAN=$f step bench_fan${f}_syn 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary --layouts synthetic; done ;;
    ptrain) step probe_train 600 python tools/probe_train.py ;;
    aseq) step probe_arch_seq 300 python tools/probe_arch_seq.py ;;
    preab) L=$PWD/rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd/heist_amd
           for i in 1 2; do step probe_policy_pre7_$i 300 python tools/probe_policy.py
             for pre in 10 13; do HEIST_LIB=$L/libheist_hip_pre$pre.so step probe_policy_pre${pre}_$i 300 python tools/probe_policy.py; done; done ;;
    lbtest) step pytest_lb 600 python -u -m pytest tests/test_gpu_trainer.py -k "layout_batch or interactive or c3" -x -v --timeout 500 --timeout-method thread ;;
    mmodesw1) export HEIST_MULTI_WAVES=1; step multi_modes 300 python tools/probe_multi_modes.py
            step pmc_modes_m1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d "$OUT/pmm1" -o m --output-format csv -- python3 tools/probe_multi_modes.py
            step pmc_modes_m2 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d "$OUT/pmm2" -o m --output-format csv -- python3 tools/probe_multi_modes.py
            python tools/pmc_summary.py "$(find "$OUT/pmm1" -name "*counter_collection.csv" | head -n 1)" step_multi_kernel "$OUT/pmc_modes_m1.json" --modes 5 3 > /dev/null 2>&1
            python tools/pmc_summary.py "$(find "$OUT/pmm2" -name "*counter_collection.csv" | head -n 1)" step_multi_kernel "$OUT/pmc_modes_m2.json" --modes 5 3 > /dev/null 2>&1; unset HEIST_MULTI_WAVES; true ;;
    mmodes) step multi_modes 300 python tools/probe_multi_modes.py
            step pmc_modes_m1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d "$OUT/pmm1" -o m --output-format csv -- python3 tools/probe_multi_modes.py
            step pmc_modes_m2 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d "$OUT/pmm2" -o m --output-format csv -- python3 tools/probe_multi_modes.py
            python tools/pmc_summary.py "$(find "$OUT/pmm1" -name "*counter_collection.csv" | head -n 1)" step_multi_kernel "$OUT/pmc_modes_m1.json" --modes 5 3 > /dev/null 2>&1
            python tools/pmc_summary.py "$(find "$OUT/pmm2" -name "*counter_collection.csv" | head -n 1)" step_multi_kernel "$OUT/pmc_modes_m2.json" --modes 5 3 > /dev/null 2>&1; true ;;
    benchtest) step pytest_bench 900 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 800 --timeout-method thread ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o heist --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary ;;
    pmc) step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o heist --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary
         step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o heist --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary ;;
    probe) step probe 600 python tools/probe_step.py ;;
    ptest) step pytest_policy 600 python -m pytest tests/test_gpu_policy.py -x -q ;;
    pprobe) step probe_policy 600 python tools/probe_policy.py ;;
    tprobe) step probe_train 600 python tools/probe_train.py ;;
    pstamp) PROBE_STAMPS=1 step policy_stamps 300 python tools/probe_policy.py ;;
    sstamp) step step_stamps 300 python tools/probe_step_stamps.py ;;
    sstampsyn) PROBE_LAYOUTS=synthetic step step_stamps_syn 300 python tools/probe_step_stamps.py ;;
    mprobesyn) PROBE_LAYOUTS=synthetic step probe_modes_syn 600 python tools/probe_step_modes.py ;;
    uprobe) step probe_update 600 python tools/probe_update.py ;;
    mprobe) step probe_modes 600 python tools/probe_step_modes.py ;;
    oprobe) step probe_obs_store 300 python tools/probe_obs_store.py ;;
    prprobe) PROBE_VAR=HEIST_STEP_PRIO PROBE_POLICIES=0,1,2,3 step probe_step_prio 300 python tools/probe_obs_store.py ;;
    sprobe) PROBE_VAR=HEIST_SPLIT_OBS PROBE_POLICIES=${PROBE_POLICIES:-0,1} step probe_split_obs 300 python tools/probe_obs_store.py ;;
    dprobe) PROBE_VAR=HEIST_DISPATCH_ORDER PROBE_POLICIES=0,1 step probe_dispatch_order 300 python tools/probe_obs_store.py ;;
    vprobe) step probe_variants 600 python tools/probe_step_variants.py ;;
    envtest) step pytest_env 900 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread ;;
    kprobe) HIP_FORCE_DEV_KERNARG=0 step bench_kernarg0 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary
            HIP_FORCE_DEV_KERNARG=1 step bench_kernarg1 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary
            step bench_kernargdef 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary ;;
    quick) step bench_quick 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary ;;
    quicksyn) step bench_quick_syn 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-secondary --layouts synthetic ;;
    ppmc) for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" \
                     "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16"; do
            i=$((i+1)); PROBE_N=4096 step pmc_policy$i 600 rocprofv3 --pmc $grp --kernel-include-regex solver_conv -d "$OUT/pp$i" -o pol --output-format csv -- python3 tools/probe_policy.py
            python tools/pmc_summary.py "$OUT/pp$i/pol_counter_collection.csv" solver_conv "$OUT/pmc_policy$i.json" > /dev/null; rm -rf "$OUT/pp$i"
          done ;;
    icache) step pmc_icache 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVES -d "$OUT/pmc_icache" -o heist --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary ;;
    tlb) step pmc_tlb 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum -d "$OUT/pmc_tlb" -o heist --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary
         step pmc_lat 120 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum -d "$OUT/pmc_lat" -o heist --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary ;;
    list) step counters 120 rocprofv3 -L ;;
    pmcsq) step pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d "$OUT/pmc_sq" -o heist --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary
           step pmc_sq2 600 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE -d "$OUT/pmc_sq2" -o heist --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary ;;
  esac
done
echo "== all done"

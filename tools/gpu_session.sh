#!/bin/bash
# One GPU session on a gpurun box: the named steps in order, each under its own time limit,
# output in gpurun_out/$TAG/<step>.log; the session stops at the first fatal exit (time limit,
# abort, segfault) and starts no further GPU step after it.
#
#   TAG=r06a tools/gpu_session.sh pytest smoke bench prof
#
# steps:
#   pytest            the whole -m gpu suite (one process)
#   pytest=<args>     pytest on the given files / -k expression (quoted, one word), -m gpu
#   smoke             __graft_entry__.smoke()
#   bench             the driver's command: bench.py --gpus 1 --steps 20 --warmup 5
#   bench_env         the headline only: bench.py --no-secondary --no-cpu-baseline
#   prof              rocprofv3 kernel trace + stats of the headline (bench.py --no-secondary)
#   pmc               PMC passes on the headline: FETCH_SIZE, WRITE_SIZE, SQ mix (+ summaries)
#   pmc_c4            the same on BASELINE C4's env-only command (tools/probe_env_configs.py, c4)
#   pmc_c5            the same on BASELINE C5's (2048 envs of 32 x 32)
#   train             tools/probe_train.py (the fp32 training iteration's parts)
#   prof_train        rocprofv3 kernel stats of tools/probe_train.py
#   arch              tools/probe_arch_update.py (Architect update kernel, per-update time)
#   configs           tools/probe_env_configs.py (env-only lines of every BASELINE config)
#   py=<script>       python3 <script> (any probe under tools/)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
TAG=${TAG:-session}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "$OUT/$name.log"
  if fatal $rc; then echo "== fatal exit $rc: session stops"; exit $rc; fi
  return 0
}
B="bench.py --no-cpu-baseline --no-secondary"
PT="python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread"
for step in "$@"; do
  case "$step" in
    pytest) run pytest_gpu 1100 $PT -q tests ;;
    pytest=*) run "pytest_$(echo "${step#pytest=}" | tr -c 'A-Za-z0-9_' '_' | cut -c1-40)" 900 $PT ${step#pytest=} ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench_env) run bench_env 300 python3 $B --steps 20 --warmup 5 ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o heist --output-format csv -- python3 $B --steps 300 --warmup 30 ;;
    pmc)
      run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o heist --output-format csv -- python3 $B --steps 100 --warmup 10
      run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o heist --output-format csv -- python3 $B --steps 100 --warmup 10
      run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$OUT/pmc_sq" -o heist --output-format csv -- python3 $B --steps 100 --warmup 10
      python tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --ticks 20 --profile "$TAG" --out "$OUT/traffic.json" > /dev/null
      python tools/pmc_sq.py "$OUT/pmc_sq" --ticks 20 --out "$OUT/pmc_sq.json" > /dev/null ;;
    pmc_c4)  # the same three passes on BASELINE C4's env-only command (8192 envs, budget 40)
      export PROBE_CONFIGS=c4
      C4="python3 tools/probe_env_configs.py"
      run pmc_c4_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_c4_fetch" -o heist --output-format csv -- $C4
      run pmc_c4_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_c4_write" -o heist --output-format csv -- $C4
      run pmc_c4_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$OUT/pmc_c4_sq" -o heist --output-format csv -- $C4
      unset PROBE_CONFIGS
      python tools/pmc_traffic.py "$OUT/pmc_c4_fetch" "$OUT/pmc_c4_write" --ticks 20 --envs 8192 --workload c4 --profile "$TAG" --out "$OUT/c4_traffic.json" > /dev/null
      python tools/pmc_sq.py "$OUT/pmc_c4_sq" --ticks 20 --out "$OUT/c4_pmc_sq.json" > /dev/null ;;
    pmc_c5)  # the same three passes on BASELINE C5's env-only command (2048 envs of 32 x 32, two waves per env)
      export PROBE_CONFIGS=c5
      C5="python3 tools/probe_env_configs.py"
      run pmc_c5_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_c5_fetch" -o heist --output-format csv -- $C5
      run pmc_c5_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_c5_write" -o heist --output-format csv -- $C5
      run pmc_c5_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$OUT/pmc_c5_sq" -o heist --output-format csv -- $C5
      unset PROBE_CONFIGS
      python tools/pmc_traffic.py "$OUT/pmc_c5_fetch" "$OUT/pmc_c5_write" --ticks 20 --envs 2048 --workload c5 --profile "$TAG" --out "$OUT/c5_traffic.json" > /dev/null
      python tools/pmc_sq.py "$OUT/pmc_c5_sq" --ticks 20 --out "$OUT/c5_pmc_sq.json" > /dev/null ;;
    train) run train 600 python3 tools/probe_train.py ;;
    prof_train) run prof_train 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_train" -o train --output-format csv -- python3 tools/probe_train.py ;;
    arch) run arch 300 python3 tools/probe_arch_update.py ;;
    configs) run configs 600 python3 tools/probe_env_configs.py ;;
    py=*) s=${step#py=}; run "py_$(basename "$s" .py)" 600 python3 $s ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all done"

#!/bin/bash
# Lean kernel: solver cell patched in registers (one store per quad); store-policy A/B
# (HEIST_OBS_STORE 2 nt default, 0 plain, 1 sc1, 3 sc1 nt), full kernel and stores-only floor.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05u}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-100; if fatal $rc; then exit $rc; fi; }
run pytest_env 900 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 300 --timeout-method thread -k "multi or lean or stamp or interval or golden or store"
for i in 1 2; do
  for pol in 2 0 1 3; do
    HEIST_OBS_STORE=$pol PROBE_LAYOUTS=architect run arch_pol${pol}_$i 300 python3 tools/probe_lean_modes.py
    HEIST_OBS_STORE=$pol HEIST_PROBE_MODE=27 PROBE_LAYOUTS=architect run floor_pol${pol}_$i 300 python3 tools/probe_lean_modes.py
  done
  PROBE_LAYOUTS=synthetic run syn_$i 300 python3 tools/probe_lean_modes.py
done
echo "== all done"

#!/bin/bash
# Lean kernel floor ladder (timing only): 27 stores alone, 28 move/patrol + stores,
# 23 everything but the obs stores, 0 the product kernel; both layouts.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05t}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-100; if fatal $rc; then exit $rc; fi; }
for i in 1 2; do
  for m in 0 27 29 30; do
    for L in architect; do
      HEIST_PROBE_MODE=$m PROBE_LAYOUTS=$L run ${L}_m${m}_$i 300 python3 tools/probe_lean_modes.py
    done
  done
done
echo "== all done"

#!/bin/bash
# Lean kernel phase costs by removal (HEIST_PROBE_MODE 21 no DMA wait, 22 no cast, 23 no obs
# stores; timings only): headline and synthetic env-only.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05p}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-150; if fatal $rc; then exit $rc; fi; }
B="bench.py --no-cpu-baseline --no-secondary --extra-windows 2 --steps 300 --warmup 30"
for i in 1 2; do
  for m in 0 21 22 23; do
    for L in architect synthetic; do
      HEIST_PROBE_MODE=$m PROBE_LAYOUTS=$L run ${L}_m${m}_$i 300 python3 tools/probe_lean_modes.py
    done
  done
done
echo "== all done"

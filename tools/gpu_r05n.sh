#!/bin/bash
# Lean stamps at 1024 / 2048 / 4096 synthetic envs (1, 2, 4 waves per SIMD): a heavy env's
# lifetime alone on its SIMD vs shared.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05n}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-150; if fatal $rc; then exit $rc; fi; }
for n in 1024 2048 4096; do
  HEIST_MULTI_WAVES=1 PROBE_N=$n PROBE_LAYOUTS=synthetic PROBE_DUMP=$OUT/syn_n$n run stamps_syn_n$n 300 python3 tools/probe_multi_stamps.py
done
echo "== all done"

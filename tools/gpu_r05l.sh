#!/bin/bash
# Raw lean stamps (per env: segments, lifetime, start, HW_ID, XCC_ID) for dispatch orders
# 0 / 1 / 2, synthetic and architect layouts: SIMD placement and per-SIMD load.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05l}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 $OUT/$name.log | cut -c1-200; if fatal $rc; then exit $rc; fi; }
for o in 0 1 2; do
  HEIST_DISPATCH_ORDER=$o PROBE_LAYOUTS=synthetic PROBE_DUMP=$OUT/syn_o$o run stamps_syn_o$o 300 python3 tools/probe_multi_stamps.py
  HEIST_DISPATCH_ORDER=$o PROBE_DUMP=$OUT/arch_o$o run stamps_arch_o$o 300 python3 tools/probe_multi_stamps.py
done
echo "== all done"

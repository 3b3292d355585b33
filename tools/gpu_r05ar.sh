#!/bin/bash
# Timing-only A/B: the lean kernel without its inlined generic fallback (HEIST_LEAN_NO_GENERIC
# variant; every env of these workloads is lean-eligible) vs the product build.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05ar}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-110; if fatal $rc; then exit $rc; fi; }
for i in 1 2; do
  for v in prod noinl nogen; do
    L=""; [ $v != prod ] && L=$PWD/tools/variants/libheist_hip_$v.so
    for lay in architect synthetic; do
      HEIST_LIB=$L PROBE_LAYOUTS=$lay run ${v}_${lay}_$i 200 python3 tools/probe_lean_modes.py
    done
  done
done
echo "== all done"

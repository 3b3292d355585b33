#!/bin/bash
# Backbone kernel: event timing forms vs rocprof's kernel durations, product vs previous build.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05ax}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 $OUT/$name.log | cut -c1-300; if fatal $rc; then exit $rc; fi; }
for v in prod polbase; do
  L=""; [ $v != prod ] && L=$PWD/tools/bin/libheist_hip_$v.so
  HEIST_LIB=$L run ev_$v 120 python3 tools/probe_backbone_kernel.py
  HEIST_LIB=$L run prof_$v 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- python3 tools/probe_backbone_kernel.py
done
echo "== all done"

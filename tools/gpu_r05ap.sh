#!/bin/bash
# A/B: heist_env.hip scheduler flags (tools/build_variant.sh: ilp = -amdgpu-sched-strategy=max-ilp,
# bias0 = -amdgpu-schedule-metric-bias=0, trk = -amdgpu-use-amdgpu-trackers) vs the product.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05ap}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-110; if fatal $rc; then exit $rc; fi; }
for i in 1 2; do
  for v in prod ilp bias0 trk; do
    L=""; [ $v != prod ] && L=$PWD/tools/variants/libheist_hip_$v.so
    for lay in architect synthetic; do
      HEIST_LIB=$L PROBE_LAYOUTS=$lay run ${v}_${lay}_$i 200 python3 tools/probe_lean_modes.py
    done
  done
done
echo "== all done"

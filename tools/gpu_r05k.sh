#!/bin/bash
# PC sampling (host trap) of step_lean_kernel on the synthetic and the headline workload.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05k}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 $OUT/$name.log | cut -c1-300; if fatal $rc; then exit $rc; fi; }
run list 60 rocprofv3 -L
grep -i -A12 "pc.sampl\|PC Sampling" $OUT/list.log | head -60
PROBE_LAYOUTS=synthetic PROBE_LAUNCHES=100 run pcs_syn 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --kernel-include-regex step_lean -d $OUT/pcs_syn -o pcs --output-format csv -- python3 tools/probe_lean_run.py
ls -R $OUT/pcs_syn | head
echo "== all done"

#!/bin/bash
# Backbone launch cost vs envs per workgroup (direct C-ABI timing): fixed per-launch cost.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05az}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 env PROBE_N=256,512,1024,2048,4096,8192,16384 python3 tools/probe_backbone_kernel.py > $OUT/sweep.log 2>&1; echo rc=$?
cat $OUT/sweep.log | grep '^{'

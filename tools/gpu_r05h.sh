#!/bin/bash
# MIOpen solver choice for the training convolutions: NHWC vs NCHW, immediate mode vs Find.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05h}
mkdir -p $OUT/miopen
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=$OUT/miopen MIOPEN_CUSTOM_CACHE_DIR=$OUT/miopen
cp miopen_cache/* $OUT/miopen/ 2>/dev/null
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 5 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
run conv_layouts 1000 python3 -u tools/probe_conv_layouts.py
echo "== all done"

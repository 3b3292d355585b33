#!/bin/bash
# Env configs x4 (synthetic / C4 / C5 spread) on one box.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05ab}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 $OUT/$name.log | cut -c1-120; if fatal $rc; then exit $rc; fi; }
for i in 1 2 3 4; do run configs_$i 600 python3 tools/probe_env_configs.py; done
echo "== all done"

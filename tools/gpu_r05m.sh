#!/bin/bash
# A/B: lean K-tick wave priority by cost rank (HEIST_PRIO_MODE 0..3): env configs and the
# headline, alternating; then the stamps of the best mode.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05m}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 $OUT/$name.log | cut -c1-200; if fatal $rc; then exit $rc; fi; }
B="bench.py --no-cpu-baseline --no-secondary --extra-windows 4 --steps 300 --warmup 30"
for i in 1 2; do
  for m in 0 1 2 3; do
    HEIST_PRIO_MODE=$m run configs_p${m}_$i 600 python3 tools/probe_env_configs.py
    HEIST_PRIO_MODE=$m run arch_p${m}_$i 300 python3 $B
  done
done
for m in 1 2; do
  HEIST_PRIO_MODE=$m PROBE_LAYOUTS=synthetic PROBE_DUMP=$OUT/syn_p$m run stamps_syn_p$m 300 python3 tools/probe_multi_stamps.py
done
echo "== all done"

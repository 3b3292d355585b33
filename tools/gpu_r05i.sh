#!/bin/bash
# A/B: heist_env.hip built with machine LICM (tools/variants/libheist_hip_licm.so) vs the
# product build: env configs and the headline, twice each, alternating.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-r05i}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 $OUT/$name.log | cut -c1-300; if fatal $rc; then exit $rc; fi; }
B="bench.py --no-cpu-baseline --no-secondary --extra-windows 4 --steps 300 --warmup 30"
V=$PWD/tools/variants/libheist_hip_licm.so
for i in 1 2; do
  run configs_prod_$i 600 python3 tools/probe_env_configs.py
  HEIST_LIB=$V run configs_licm_$i 600 python3 tools/probe_env_configs.py
  run arch_prod_$i 300 python3 $B
  HEIST_LIB=$V run arch_licm_$i 300 python3 $B
done
HEIST_LIB=$V run pytest_licm 900 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 300 --timeout-method thread -k "multi or lean"
echo "== all done"

#!/bin/bash
# A/B of a compile-time variant of the library: the default build against the one named by
# ALT_LIB (e.g. built with an extra -D), alternating quick bench runs in separate processes
# (HEIST_LIB selects the library a process loads).  r02bk compared a head that forced every
# kernel argument into SGPRs at entry (16.41 us) with the default head (16.17 us).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
for i in 1 2 3; do
  for v in default alt; do
    if [ $v = alt ]; then export HEIST_LIB=$PWD/$ALT_LIB; else unset HEIST_LIB; fi
    timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-secondary > $OUT/$v.$i.log 2>&1 || exit $?
    echo "$v $i $(grep -o '"kernel_ms": [0-9.]*' $OUT/$v.$i.log)"
  done
done

#!/bin/bash
# Does ROCm's SLP vectorizer still break the fast raycast?  heist_env.hip builds with
# -fno-slp-vectorize (heist_amd/_build.py): ROCm 7.2 clang's packed-fp32 (v_pk_*_f32) forms
# of the raycast lost a lane's negation (march_fast) and merged the two tie-table lookups
# (near_tie).  This runs the raycast parity tests against a library built from the same
# sources WITHOUT the flag (tools/forensic/slp_build/libheist_hip_slp.so, made by
#   HEIST_LIB=$PWD/tools/forensic/slp_build/libheist_hip_slp.so \
#   HEIST_ENV_FLAGS="-mllvm -disable-machine-licm" python -c "...; _build.build(force=True)"
# on the build host) and counts the packed-fp32 instructions in both builds' heist_env code.
# A failing parity run = the miscompile persists and the flag is still needed; all green =
# the flag can be dropped (then also drop this script).  The suite's own check that would
# catch the bug in the product build is tests/test_gpu_env.py::test_cones_fast_equals_exact
# (fast path against the exact path, every direction quadrant) with the golden traces.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${TAG:-forensic}
mkdir -p $OUT
export TMPDIR=/tmp
LIB=tools/forensic/slp_build/libheist_hip_slp.so
[ -f $LIB ] || { echo "missing $LIB"; exit 1; }
# llvm-objdump --offloading only EXTRACTS the device bundles (next to the input file), so
# extract from a copy in a scratch directory and disassemble the gfx950 objects
for f in rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd/heist_amd/libheist_hip.so $LIB; do
  d=$(mktemp -d) && cp "$f" $d/lib.so && (cd $d && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading lib.so > /dev/null 2>&1)
  n=0
  for o in $d/lib.so.*gfx950; do
    /opt/rocm/lib/llvm/bin/llvm-readelf -s "$o" 2>/dev/null | grep -q step_lean_kernel || continue  # heist_env.hip's object
    # v_pk_fma_f32 also comes from the raycast's one deliberate inline-asm packed FMA
    n=$(/opt/rocm/lib/llvm/bin/llvm-objdump -d "$o" | grep -o "v_pk_[a-z]*_f32" | sort | uniq -c | tr -s ' \n' ' ')
  done
  echo "$f: packed-fp32 instructions in heist_env's device code: $n" | tee -a $OUT/slp_isa_counts.txt
  rm -rf $d
done
HEIST_LIB=$PWD/$LIB timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -m gpu -q --timeout 300 \
  --timeout-method thread -k "golden_trace or cones_bit_exact or cones_fast_equals_exact or fast_direction or full_size_sampled" \
  > $OUT/slp_parity.log 2>&1
echo "parity without -fno-slp-vectorize: rc=$?"; tail -n 5 $OUT/slp_parity.log

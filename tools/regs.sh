#!/bin/bash
# Register / occupancy / spill report of the env kernels (cross-compiled for gfx950, no GPU).
# usage: tools/regs.sh [regex]   (default: step|reset|cones)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$ROOT/rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd/csrc
OUT=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math ${HEIST_ENV_FLAGS:--fno-slp-vectorize -mllvm -disable-machine-licm} --offload-arch=gfx950 \
  -I "$ROOT/include" -I "$CSRC" -c "$CSRC/heist_env.hip" -o "$OUT/he.o" -Rpass-analysis=kernel-resource-usage \
  > "$OUT/res.txt" 2>&1 || { grep -E "error" "$OUT/res.txt" | head -20; exit 1; }
grep -E "remark: +(Function Name|VGPRs:|Occupancy|VGPRs Spill)" "$OUT/res.txt" | sed 's/.*remark: *//; s/ \[-Rpass.*//' \
  | paste - - - - | sed 's/Function Name: _ZN5heist//; s/EEEvNS[^\t]*//' | grep -E "${1:-step|reset|cones}"
rm -rf "$OUT"

#!/bin/bash
# A/B build of one source with other flags, linked with the product's other objects into
# tools/variants/libheist_hip_<name>.so (load it with HEIST_LIB=...); the product build and
# its objects are untouched.
#   usage: tools/build_variant.sh <name> "<flags>" [source, default heist_env.hip]
# (the flags replace the source's product-only ones: for heist_env.hip pass
# "-fno-slp-vectorize -mllvm -disable-machine-licm" plus the variant's own.)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd
NAME=$1; FLAGS=$2; SRC=${3:-heist_env.hip}; REPL=${4:-${SRC%.hip}}  # 4th: the product object it replaces
STEM=${SRC%.hip}
OUT=$ROOT/tools/variants; mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function --offload-arch=gfx950 \
  -I $ROOT/include -I $PKG/csrc $FLAGS -c $PKG/csrc/$SRC -o $OUT/${STEM}_$NAME.o
TL=$(python3 -c "import torch,os; print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
OBJS=$(ls $PKG/build/*.o | grep -v "/$REPL.o$")
g++ -shared -o $OUT/libheist_hip_$NAME.so $OUT/${STEM}_$NAME.o $OBJS -L$TL -l:libamdhip64.so -Wl,-rpath,$TL
rm -f $OUT/${STEM}_$NAME.o
echo $OUT/libheist_hip_$NAME.so

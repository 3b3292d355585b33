#!/bin/bash
# A/B build of heist_env.hip with other flags, linked with the product's other objects into
# tools/variants/libheist_hip_<name>.so (load it with HEIST_LIB=...); the product build and
# its objects are untouched.   usage: tools/build_variant.sh <name> "<heist_env.hip flags>"
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd
NAME=$1; FLAGS=$2
OUT=$ROOT/tools/variants; mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function --offload-arch=gfx950 \
  -I $ROOT/include -I $PKG/csrc $FLAGS -c $PKG/csrc/heist_env.hip -o $OUT/heist_env_$NAME.o
TL=$(python3 -c "import torch,os; print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
OBJS=$(ls $PKG/build/*.o | grep -v heist_env.o)
g++ -shared -o $OUT/libheist_hip_$NAME.so $OUT/heist_env_$NAME.o $OBJS -L$TL -l:libamdhip64.so -Wl,-rpath,$TL
rm -f $OUT/heist_env_$NAME.o
echo $OUT/libheist_hip_$NAME.so

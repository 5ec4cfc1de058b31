#!/bin/bash
# Build an alternative libasrx.so for A/B timing: tools/exp/build_variant.sh <name> <source.hip> [flags]
# The variant source replaces the production object of the same basename (csrc/<base>.hip);
# every other object is the production one from asr-model_amd/build.
set -e
SRC_ABS=$(realpath "$2")
cd "$(dirname "$0")/../../asr-model_amd"
NAME=$1; SRC=$SRC_ABS; shift 2
BASE=$(basename "$SRC" .hip); BASE=${BASE%_old}; BASE=${BASE%_v2}
mkdir -p ../tools/exp/vbuild
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Icsrc "$@" -c "$SRC" -o ../tools/exp/vbuild/${BASE}_$NAME.o
OBJS=$(ls build/*.o | grep -v "build/$BASE.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS ../tools/exp/vbuild/${BASE}_$NAME.o -o ../tools/exp/libasrx_$NAME.so
echo built tools/exp/libasrx_$NAME.so from $SRC replacing $BASE

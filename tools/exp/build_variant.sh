#!/bin/bash
# Build an alternative libasrx.so for A/B timing: tools/exp/build_variant.sh <name> <gemm_wn source> [extra flags]
# (every other object is the production one from asr-model_amd/build).
set -e
cd "$(dirname "$0")/../../asr-model_amd"
NAME=$1; SRC=$2; shift 2
mkdir -p ../tools/exp/vbuild
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Icsrc "$@" -c "$SRC" -o ../tools/exp/vbuild/gemm_wn_$NAME.o
OBJS=$(ls build/*.o | grep -v gemm_wn.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS ../tools/exp/vbuild/gemm_wn_$NAME.o -o ../tools/exp/libasrx_$NAME.so
echo built tools/exp/libasrx_$NAME.so

#!/bin/bash
# A/B build of the weight-stationary GEMM: gemm_ws_{a,b,c}.hip and gemm_wn.hip recompiled with extra flags
# (e.g. -DWS_BK=32), linked with the production objects of everything else -> tools/exp/libasrx_<name>.so
# (load it with ASRX_LIB=...).  usage: tools/exp/build_ws_variant.sh <name> [flags...]
set -e
cd "$(dirname "$0")/../../asr-model_amd"
NAME=$1; shift
D=../tools/exp/vbuild/$NAME; mkdir -p $D
for f in csrc/gemm_ws_a.hip csrc/gemm_ws_b.hip csrc/gemm_ws_c.hip csrc/gemm_wn.hip; do
  b=$(basename $f .hip)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Icsrc "$@" -c $f -o $D/$b.o &
done
wait
OBJS=$(ls build/*.o | grep -v -E "build/gemm_ws_|build/gemm_wn.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $D/*.o -o ../tools/exp/libasrx_$NAME.so
echo built tools/exp/libasrx_$NAME.so

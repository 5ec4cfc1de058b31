#!/bin/bash
# A/B build of the wide GEMM: every gemm_wr_* unit recompiled with extra flags (e.g. -DWR_DEPTH=4),
# linked with the production objects of everything else -> tools/exp/libasrx_<name>.so (load it with
# ASRX_LIB=...).  usage: tools/exp/build_wr_variant.sh <name> [flags...]
set -e
cd "$(dirname "$0")/../../asr-model_amd"
NAME=$1; shift
D=../tools/exp/vbuild/$NAME; mkdir -p $D
for f in csrc/gemm_wr_*.hip; do
  b=$(basename $f .hip)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Icsrc "$@" -c $f -o $D/$b.o &
done
wait
OBJS=$(ls build/*.o | grep -v "build/gemm_wr_")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $D/*.o -o ../tools/exp/libasrx_$NAME.so
echo built tools/exp/libasrx_$NAME.so

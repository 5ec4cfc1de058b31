#!/bin/bash
# GPU call: kernel times (rocprofv3 --kernel-trace --stats) and one SQ counter pass of the log-mel
# microbench (tools/microbench.py mel) for the production library and optional variants.
# usage: tools/exp/melprof.sh TAG [variant.so ...]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for v in prod "$@"; do
  if [ $v = prod ]; then L=""; else L=$R/tools/exp/libasrx_$v.so; fi
  ASRX_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/melk_${TAG}_$v -o run --output-format csv -- python3 $R/tools/microbench.py mel > $R/gpurun_out/melk_${TAG}_$v.log 2>&1
  ASRX_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $R/gpurun_out/melq_${TAG}_$v -o run --output-format csv -- python3 $R/tools/microbench.py mel > $R/gpurun_out/melq_${TAG}_$v.log 2>&1
  echo "== $v"; grep -h logmel $R/gpurun_out/melk_${TAG}_$v.log
done
echo melprof-ok

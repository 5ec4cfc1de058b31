#!/bin/bash
# GPU call: SQ issue / wait counters (one pass, 8 SQ + GRBM_GUI_ACTIVE) over isolated launches of the wide GEMM
# (tools/gemm_micro.py subset) and the AbbyNormal row kernels (tools/microbench.py abby), plus the counter list.
# usage: tools/gpu_sq_pmc.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc_list_$TAG.txt 2>&1 || true
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
GEMM_SHAPES="192064,384,384;192064,384,1536;192064,1536,384" GEMM_NJ=3 GEMM_ITERS=5 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $R/gpurun_out/sqg_$TAG -o run --output-format csv -- python3 $R/tools/gemm_micro.py > $R/gpurun_out/sqg_$TAG.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $R/gpurun_out/sqa_$TAG -o run --output-format csv -- python3 $R/tools/microbench.py abby > $R/gpurun_out/sqa_$TAG.log 2>&1
echo sq-ok

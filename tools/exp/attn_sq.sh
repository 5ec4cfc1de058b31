#!/bin/bash
# SQ issue / wait counters (one pass) over the attention A/B microbench (tools/exp/attn_ab.py)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $R/gpurun_out/attn_sq -o run --output-format csv -- python3 $R/tools/exp/attn_ab.py > $R/gpurun_out/attn_sq.log 2>&1
C2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_WAVE32_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/attn_sq2 -o run --output-format csv -- python3 $R/tools/exp/attn_ab.py > $R/gpurun_out/attn_sq2.log 2>&1 || echo "pass2 failed"
echo attn-sq-ok

#!/bin/bash
# GPU call: attention forward kernel variants (ASRX_ATTN_VARIANT 0..7), one process each.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 3 4 5 6 7}; do
  ASRX_ATTN_VARIANT=$v timeout -k 10 120 python tools/microbench.py attnf >> gpurun_out/attn_variants.log 2>&1
done
cat gpurun_out/attn_variants.log | grep variant

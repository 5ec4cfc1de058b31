#!/bin/bash
# Software-pipelined attention forward: bit-identity tests, then A/B micro (variant 1 vs 0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_sp.py > gpurun_out/r05_w_tests.log 2>&1 || { tail -40 gpurun_out/r05_w_tests.log; exit 1; }
tail -3 gpurun_out/r05_w_tests.log
O=gpurun_out/r05_w_micro.txt
: > $O
for v in 0 1 0 1; do
  echo "== ATTN_VARIANT=$v" >> $O
  ATTN_VARIANT=$v timeout -k 10 300 python -u tools/attn_micro.py 1 >> $O 2>&1 || exit 1
done
cat $O

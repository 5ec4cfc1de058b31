#!/bin/bash
# GPU call: GEMM parity tests + GEMM microbench.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or wide or conv or router or abby or linear" > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
timeout -k 10 200 python tools/microbench.py gemm > gpurun_out/gemm_mb.log 2>&1
grep -v Warn gpurun_out/gemm_mb.log | head -60

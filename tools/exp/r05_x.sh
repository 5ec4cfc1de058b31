#!/bin/bash
# router64_kernel: bit-identity tests, then A/B micro.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_router64.py tests/test_gpu_gemm_mel.py > gpurun_out/r05_x_tests.log 2>&1 || { tail -40 gpurun_out/r05_x_tests.log; exit 1; }
tail -3 gpurun_out/r05_x_tests.log
timeout -k 10 300 python -u tools/router_micro.py > gpurun_out/r05_x_micro.txt 2>&1 || { cat gpurun_out/r05_x_micro.txt; exit 1; }
cat gpurun_out/r05_x_micro.txt

#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_lt.py tests/test_gpu_model.py tests/test_gpu_msheath_composite.py -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/r06_n_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r06_n_tests.log | tail -12; [ $rc -eq 0 ] || exit 1
SKIPTEST=1 TAG=r06_n bash tools/r06_d.sh

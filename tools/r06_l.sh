#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_msheath_composite.py tests/test_gpu_model.py tests/test_gpu_bf16_storage.py tests/test_gpu_gemm_p2.py tests/test_gpu_fusions.py tests/test_gpu_rot_fused.py tests/test_gpu_ce_fused.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r06_l_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_l_tests.log; [ $rc -eq 0 ] || exit 1
SKIPTEST=1 TAG=r06_l bash tools/r06_d.sh

#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msheath_composite.py tests/test_gpu_gemm_lt.py tests/test_gpu_gemm_p2.py 2>&1 | tail -3 || exit 1
timeout -k 10 400 python -u bench.py --config small --batch 8 --steps 6 --warmup 2 --no-fp32-line --no-cpu-baseline --no-refpitch-line --no-dead-block-line > gpurun_out/r06_small_nj.json 2>gpurun_out/r06_small_nj.err || exit 1
cut -c1-400 gpurun_out/r06_small_nj.json
timeout -k 10 400 python -u bench.py --config medium --batch 8 --steps 3 --warmup 2 --no-fp32-line --no-cpu-baseline --no-refpitch-line --no-dead-block-line --no-probe > gpurun_out/r06_medium_nj.json 2>gpurun_out/r06_medium_nj.err || exit 1
cut -c1-400 gpurun_out/r06_medium_nj.json

#!/bin/bash
# MSheath per-call workspaces: tests, then the small-config line (host-bound) and the headline line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_fusions.py tests/test_gpu_gemm_mel.py tests/test_gpu_model_configs.py > gpurun_out/r05_ae_tests.log 2>&1 || { tail -30 gpurun_out/r05_ae_tests.log; exit 1; }
tail -2 gpurun_out/r05_ae_tests.log
timeout -k 10 600 python -u bench.py --config small --batch 8 --no-cpu-baseline --no-refpitch-line --no-dead-block-line > gpurun_out/r05_ae_small.json 2> gpurun_out/r05_ae_small.err || { tail -20 gpurun_out/r05_ae_small.err; exit 1; }
cut -c1-200 gpurun_out/r05_ae_small.json
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-refpitch-line --no-dead-block-line > gpurun_out/r05_ae_tiny.json 2> gpurun_out/r05_ae_tiny.err || { tail -20 gpurun_out/r05_ae_tiny.err; exit 1; }
cut -c1-200 gpurun_out/r05_ae_tiny.json

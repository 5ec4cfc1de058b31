#!/bin/bash
# x_new + mem column sums with 8 rows per trip: MSheath tests, the dead-block schedule test (printed gap /
# spread), then a kernel-trace profile of the headline step (axpy_row2_colsum average vs 29.5 us).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "msheath or axpy or mem" > gpurun_out/r05_af_tests.log 2>&1 || { tail -30 gpurun_out/r05_af_tests.log; exit 1; }
tail -1 gpurun_out/r05_af_tests.log
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_model.py > gpurun_out/r05_af_model.log 2>&1 || { tail -30 gpurun_out/r05_af_model.log; exit 1; }
grep -E "rerun spread|schedule gap" gpurun_out/r05_af_model.log; tail -1 gpurun_out/r05_af_model.log
bash tools/gpu_prof.sh r05_af

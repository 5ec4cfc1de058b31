#!/bin/bash
# GPU call: GEMM parity tests, wgrad split-K sweep, FETCH_SIZE pass over one wgrad shape.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or wide or conv or router or linear or wgrad" > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
timeout -k 10 120 python tools/wgrad_sweep.py > gpurun_out/ws2.log 2>&1
grep -v amdgpu.ids gpurun_out/ws2.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/wpmc3 -o run --output-format csv -- python3 $R/tools/wgrad_one.py > $R/gpurun_out/wpmc3.log 2>&1
echo pmc-ok

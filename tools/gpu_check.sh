#!/bin/bash
# One GPU call: gpu parity tests, default bench line, rocprofv3 kernel stats of the bench.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
if [ "$1" = "dist" ]; then
  timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --batch 4 --dist-backend gloo --same-device --no-cpu-baseline --no-optimizer > gpurun_out/bench_dist2.json 2> gpurun_out/bench_dist2.err || { tail -30 gpurun_out/bench_dist2.err; exit 1; }
  cat gpurun_out/bench_dist2.json
fi
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
if [ "$1" = "prof" ]; then bash tools/prof3.sh; fi

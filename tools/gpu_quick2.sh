#!/bin/bash
# GPU call: GEMM/model GPU tests + bench line.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k "gemm or model or msheath or generate" > gpurun_out/t_q2.log 2>&1 || { tail -30 gpurun_out/t_q2.log; exit 1; }
tail -1 gpurun_out/t_q2.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-optimizer > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-330 gpurun_out/bench.json

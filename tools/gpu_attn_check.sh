#!/bin/bash
# GPU call: attention parity tests, attention microbench, one bench line.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k "attn or attention or generate or model" > gpurun_out/t_attn.log 2>&1 || { tail -30 gpurun_out/t_attn.log; exit 1; }
tail -2 gpurun_out/t_attn.log
timeout -k 10 200 python tools/microbench.py attn > gpurun_out/attn_bench.log 2>&1
grep "mf \|fp8" gpurun_out/attn_bench.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-optimizer > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-330 gpurun_out/bench.json

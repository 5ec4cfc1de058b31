#!/bin/bash
# GPU call: the whole -m gpu suite, then one bench line (10 timed steps).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-optimizer > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-330 gpurun_out/bench.json

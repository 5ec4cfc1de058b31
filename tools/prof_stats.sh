#!/bin/bash
# rocprofv3 kernel stats of the bench (graph replay, 1 warmup + 3 timed = 4 steps).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof3 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe > $R/gpurun_out/prof3.log 2>&1
tail -1 $R/gpurun_out/prof3.log | cut -c1-300

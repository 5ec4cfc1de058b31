#!/bin/bash
# GPU call: the N>1 code path on one GPU -- GradSync over a 1-rank RCCL group (test + bench), next to
# the eager and graph-replay N=1 bench lines it is compared with.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 240 --timeout-method thread > gpurun_out/t_dist.log 2>&1 || { tail -30 gpurun_out/t_dist.log; exit 1; }
tail -3 gpurun_out/t_dist.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --dist-single --no-cpu-baseline --no-optimizer > gpurun_out/bench_dist_single.json 2> gpurun_out/bench_dist_single.err || { tail -30 gpurun_out/bench_dist_single.err; exit 1; }
cut -c1-400 gpurun_out/bench_dist_single.json
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --eager --no-cpu-baseline --no-optimizer --no-dead-block-line > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err || { tail -30 gpurun_out/bench_eager.err; exit 1; }
cut -c1-300 gpurun_out/bench_eager.json

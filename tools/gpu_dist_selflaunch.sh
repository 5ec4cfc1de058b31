set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_optim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_optim.log 2>&1 || { tail -30 gpurun_out/t_optim.log; exit 1; }
tail -2 gpurun_out/t_optim.log
timeout -k 10 400 python bench.py --gpus 2 --steps 2 --warmup 1 --batch 4 --dist-backend gloo --same-device --no-cpu-baseline --no-optimizer > gpurun_out/bench_dist2.json 2> gpurun_out/bench_dist2.err || { tail -30 gpurun_out/bench_dist2.err; exit 1; }
cat gpurun_out/bench_dist2.json

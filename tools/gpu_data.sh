set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_data.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_data.log 2>&1 || { tail -40 gpurun_out/t_data.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/t_data.log | tail -5
timeout -k 10 300 python tools/io_bench.py 32 > gpurun_out/io_bench.json 2> gpurun_out/io_bench.err || { tail -20 gpurun_out/io_bench.err; exit 1; }
cat gpurun_out/io_bench.json

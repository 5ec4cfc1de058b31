# round-3 GPU check: selected tests (pytest -k expression in $1, "" = the listed files), then the bench
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
FILES=${FILES:-"tests/test_gpu_bf16_storage.py tests/test_gpu_gemm_mel.py tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_model_configs.py tests/test_gpu_dist.py"}
timeout -k 10 900 python -u -m pytest $FILES -x -v --timeout 300 --timeout-method thread ${1:+-k "$1"} > gpurun_out/t_r03.log 2>&1 || { grep -E "PASSED|FAILED|Error|error" gpurun_out/t_r03.log | tail -40; tail -60 gpurun_out/t_r03.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r03.log | tail -3
if [ "$2" = "bench" ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench_r03.json 2> gpurun_out/bench_r03.err || { tail -30 gpurun_out/bench_r03.err; exit 1; }
  cat gpurun_out/bench_r03.json
fi

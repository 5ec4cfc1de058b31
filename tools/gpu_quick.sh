# one GPU call: selected tests (args = pytest -k expression), then the default bench line
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$1" > gpurun_out/t_quick.log 2>&1 || { tail -60 gpurun_out/t_quick.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED|passed|failed" gpurun_out/t_quick.log | tail -30
if [ "$2" = "bench" ]; then
  timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi

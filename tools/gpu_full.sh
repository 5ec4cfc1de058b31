# full GPU test suite (one process, per-test timeout) then the bench
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${1:+-k "$1"} > gpurun_out/t_full.log 2>&1 || { grep -E "PASSED|FAILED|Error|error|assert" gpurun_out/t_full.log | tail -40; exit 1; }
grep -cE "PASSED" gpurun_out/t_full.log; tail -1 gpurun_out/t_full.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['ms_per_step'],d.get('dead_block_eliminated',{}).get('value'))"

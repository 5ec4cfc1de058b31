#!/bin/bash
# round-3 GPU check: the whole -m gpu suite, smoke, then the default bench line
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
rc=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/t_r03.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|Fatal" gpurun_out/t_r03.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
grep -E "passed|failed" gpurun_out/t_r03.log | tail -2
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03.log 2>&1 || { tail -20 gpurun_out/smoke_r03.log; exit 1; }
tail -1 gpurun_out/smoke_r03.log
timeout -k 10 400 python bench.py > gpurun_out/bench_r03.json 2> gpurun_out/bench_r03.err || { tail -30 gpurun_out/bench_r03.err; exit 1; }
cat gpurun_out/bench_r03.json

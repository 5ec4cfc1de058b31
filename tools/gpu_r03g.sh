#!/bin/bash
# round-3: parity trace (where fp32 HIP leaves the oracle), re-gated tests, parity metrics, bench
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R/.snap 2>/dev/null || cd $R
timeout -k 10 300 python -u tools/parity_trace.py 2 10 64 > $O/trace_b2.log 2>&1 || { tail -20 $O/trace_b2.log; exit 1; }
grep -v Warn $O/trace_b2.log | head -5
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_storage.py tests/test_gpu_ce_fused.py "tests/test_gpu_ops.py::test_abby_normal" -v -s --timeout 200 --timeout-method thread > $O/t_r03g.log 2>&1; rc=$?
grep -E "PASSED|FAILED|worst" $O/t_r03g.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/parity_measure.py tiny_full tiny_b2 refmain > $O/parity_r03c.jsonl 2> $O/parity_r03c.err || { tail -20 $O/parity_r03c.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_r03g.json 2> $O/bench_r03g.err || { tail -30 $O/bench_r03g.err; exit 1; }
cat $O/bench_r03g.json

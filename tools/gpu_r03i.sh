#!/bin/bash
# round-3: a targeted wide-GEMM check first (the previous call aborted there), then the whole -m gpu
# suite, a rocprof kernel trace of the bench and the bench line
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
timeout -k 10 120 python -u -m pytest tests/test_gpu_bf16_storage.py -v -k "wide_gemm" --timeout 60 --timeout-method thread > $O/t_r03i_pre.log 2>&1 || { tail -30 $O/t_r03i_pre.log; exit 1; }
grep -E "passed|failed" $O/t_r03i_pre.log | tail -1
rc=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/t_r03i.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|Fatal" $O/t_r03i.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
grep -E "passed|failed" $O/t_r03i.log | tail -2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03i -o run --output-format csv -- python3 $S/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line --steps 3 --warmup 1 > $O/prof_r03i.log 2>&1 || { tail -5 $O/prof_r03i.log; exit 1; }
cd $S && timeout -k 10 400 python bench.py > $O/bench_r03i.json 2> $O/bench_r03i.err || { tail -30 $O/bench_r03i.err; exit 1; }
cat $O/bench_r03i.json

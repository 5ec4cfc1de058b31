#!/bin/bash
# round-3: wide GEMM with bias gradient fused into the weight-gradient pass -- GEMM / fusion / CE tests, GEMM micro-benchmark,
# default bench line + kernel trace
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_r03u.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|Fatal|passed|failed" $O/t_r03u.log | tail -5
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
BA="$S/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03u -o run --output-format csv -- python3 $BA --steps 3 --warmup 1 > $O/prof_r03u.log 2>&1 || { tail -5 $O/prof_r03u.log; exit 1; }
cd $S && timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_r03u.json 2> $O/bench_r03u.err || { tail -30 $O/bench_r03u.err; exit 1; }
cat $O/bench_r03u.json

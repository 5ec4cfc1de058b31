#!/bin/bash
# round-3: wide GEMM buffer-load operands + scalar tile-list read, AbbyNormal instruction cuts:
# full GPU suite, GEMM micro-benchmark (prod vs pipeline depth 4), default bench line + kernel trace
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
rc=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/t_r03o.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|Fatal" $O/t_r03o.log | head -30
grep -E "passed|failed" $O/t_r03o.log | tail -2
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u tools/gemm_micro.py > $O/gemm_micro_r03o.txt 2>&1 || { tail -5 $O/gemm_micro_r03o.txt; exit 1; }
ASRX_LIB=$S/tools/exp/libasrx_d4.so timeout -k 10 300 python -u tools/gemm_micro.py > $O/gemm_micro_r03o_d4.txt 2>&1 || { tail -5 $O/gemm_micro_r03o_d4.txt; exit 1; }
paste $O/gemm_micro_r03o.txt $O/gemm_micro_r03o_d4.txt | cut -c1-120
cd /tmp && export TMPDIR=/tmp
BA="$S/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03o -o run --output-format csv -- python3 $BA --steps 3 --warmup 1 > $O/prof_r03o.log 2>&1 || { tail -5 $O/prof_r03o.log; exit 1; }
cd $S && timeout -k 10 400 python bench.py > $O/bench_r03o.json 2> $O/bench_r03o.err || { tail -30 $O/bench_r03o.err; exit 1; }
cat $O/bench_r03o.json

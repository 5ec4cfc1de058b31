#!/bin/bash
# round-3: wide GEMM with 64-deep k-steps for nj1 -- GEMM / fusion / CE tests, GEMM micro-benchmark,
# default bench line + kernel trace
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
rc=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fusions.py tests/test_gpu_ce_fused.py tests/test_gpu_bf16_storage.py tests/test_gpu_gemm_mel.py tests/test_gpu_model_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_r03s.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|Fatal|passed|failed" $O/t_r03s.log | tail -5
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u tools/gemm_micro.py > $O/gemm_micro_r03s.txt 2>&1 || { tail -5 $O/gemm_micro_r03s.txt; exit 1; }
cat $O/gemm_micro_r03s.txt
cd /tmp && export TMPDIR=/tmp
BA="$S/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03s -o run --output-format csv -- python3 $BA --steps 3 --warmup 1 > $O/prof_r03s.log 2>&1 || { tail -5 $O/prof_r03s.log; exit 1; }
cd $S && timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_r03s.json 2> $O/bench_r03s.err || { tail -30 $O/bench_r03s.err; exit 1; }
cat $O/bench_r03s.json
timeout -k 10 400 python bench.py --config small --batch 8 --steps 3 --warmup 1 --no-cpu-baseline --no-dead-block-line --no-refpitch-line > $O/bench_r03s_small.json 2> $O/bench_r03s_small.err || { tail -20 $O/bench_r03s_small.err; exit 1; }
timeout -k 10 400 python bench.py --config medium --batch 2 --steps 3 --warmup 1 --no-cpu-baseline --no-dead-block-line --no-refpitch-line > $O/bench_r03s_medium.json 2> $O/bench_r03s_medium.err || { tail -20 $O/bench_r03s_medium.err; exit 1; }
cut -c1-200 $O/bench_r03s_small.json $O/bench_r03s_medium.json

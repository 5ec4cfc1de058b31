#!/bin/bash
# round-3: parity config tests (ulp yardstick, bf16 replay), fused-CE tests, GEMM micro-benchmark,
# bench kernel trace (CE tile order), small / medium bench lines
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
rc=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_model_configs.py tests/test_gpu_ce_fused.py -m gpu -v --timeout 400 --timeout-method thread -k "configs or ce" > $O/t_r03n.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|Fatal" $O/t_r03n.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
grep -E "passed|failed" $O/t_r03n.log | tail -2
timeout -k 10 300 python -u tools/gemm_micro.py > $O/gemm_micro_r03n.txt 2>&1 || { tail -5 $O/gemm_micro_r03n.txt; exit 1; }
cat $O/gemm_micro_r03n.txt
cd /tmp && export TMPDIR=/tmp
BA="$S/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03n -o run --output-format csv -- python3 $BA --steps 3 --warmup 1 > $O/prof_r03n.log 2>&1 || { tail -5 $O/prof_r03n.log; exit 1; }
cd $S && bash tools/gpu_r03_small.sh

#!/bin/bash
# round-3 final evidence: PMC FETCH / WRITE / MFMA-busy passes over one eager step, small / medium lines,
# whole-model parity records (decisions, replay, fp32 and ulp yardsticks)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd /tmp && export TMPDIR=/tmp
BA="$S/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmcf_r03v -o run --output-format csv -- python3 $BA --steps 1 --warmup 0 --eager > $O/pmcf_r03v.log 2>&1 || { tail -5 $O/pmcf_r03v.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmcw_r03v -o run --output-format csv -- python3 $BA --steps 1 --warmup 0 --eager > $O/pmcw_r03v.log 2>&1 || { tail -5 $O/pmcw_r03v.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $O/pmcm_r03v -o run --output-format csv -- python3 $BA --steps 1 --warmup 0 --eager > $O/pmcm_r03v.log 2>&1 || { tail -5 $O/pmcm_r03v.log; exit 1; }
echo pmc-ok
cd $S
timeout -k 10 400 python bench.py --config small --batch 8 --steps 3 --warmup 1 --no-cpu-baseline --no-dead-block-line --no-refpitch-line > $O/bench_r03v_small.json 2> $O/bench_r03v_small.err || { tail -20 $O/bench_r03v_small.err; exit 1; }
timeout -k 10 400 python bench.py --config medium --batch 2 --steps 3 --warmup 1 --no-cpu-baseline --no-dead-block-line --no-refpitch-line > $O/bench_r03v_medium.json 2> $O/bench_r03v_medium.err || { tail -20 $O/bench_r03v_medium.err; exit 1; }
cut -c1-200 $O/bench_r03v_small.json $O/bench_r03v_medium.json

#!/bin/bash
# round-3: small / medium 1-GPU bench lines (north_star's target config) + an MFMA-busy PMC pass on small
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
timeout -k 10 400 python bench.py --config small --batch 8 --steps 3 --warmup 1 --no-cpu-baseline --no-dead-block-line --no-refpitch-line > $O/bench_r03_small.json 2> $O/bench_r03_small.err || { tail -20 $O/bench_r03_small.err; exit 1; }
cat $O/bench_r03_small.json
timeout -k 10 400 python bench.py --config medium --batch 2 --steps 3 --warmup 1 --no-cpu-baseline --no-dead-block-line --no-refpitch-line > $O/bench_r03_medium.json 2> $O/bench_r03_medium.err || { tail -20 $O/bench_r03_medium.err; exit 1; }
cat $O/bench_r03_medium.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmcm_small -o run --output-format csv -- python3 $S/bench.py --config small --batch 8 --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line --steps 1 --warmup 0 --eager > $O/pmcm_small.log 2>&1 || { tail -5 $O/pmcm_small.log; exit 1; }
echo pmc-ok

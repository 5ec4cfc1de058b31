#!/bin/bash
# round 6, call c: kernel stats of the small and medium B = 8 steps (eager), and the dead-block graphs at medium
set -e
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; mkdir -p $R/gpurun_out
B="$R/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06_small -o run --output-format csv -- python3 $B --config small --batch 8 --steps 2 --warmup 1 > $R/gpurun_out/prof_r06_small.log 2>&1
tail -1 $R/gpurun_out/prof_r06_small.log | cut -c1-250
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06_medium -o run --output-format csv -- python3 $B --config medium --batch 8 --steps 1 --warmup 1 > $R/gpurun_out/prof_r06_medium.log 2>&1
tail -1 $R/gpurun_out/prof_r06_medium.log | cut -c1-250
cd $R
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line --config medium --batch 8 --steps 3 --graph-dead > gpurun_out/r06_c_medium_graph.json 2> gpurun_out/r06_c_medium_graph.err
cut -c1-300 gpurun_out/r06_c_medium_graph.json
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line --config medium --batch 8 --steps 3 > gpurun_out/r06_c_medium_eager.json 2> gpurun_out/r06_c_medium_eager.err
cut -c1-300 gpurun_out/r06_c_medium_eager.json

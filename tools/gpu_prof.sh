#!/bin/bash
# GPU call: rocprofv3 kernel trace + stats of the headline bench step (graph replay, 1 warm-up + 3 timed =
# 4 executed steps; no side lines, so every launch belongs to the headline step) and, with PMC=1,
# separate FETCH_SIZE / WRITE_SIZE passes and an MFMA-busy pass over one eager step.
# usage: tools/gpu_prof.sh TAG [bench args...]   (e.g. --config small --batch 8)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $B --steps 3 --warmup 2 > $R/gpurun_out/prof_$TAG.log 2>&1
tail -1 $R/gpurun_out/prof_$TAG.log | cut -c1-300
if [ "$PMC" = 1 ]; then
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmcf_$TAG -o run --output-format csv -- python3 $B --steps 1 --warmup 0 --eager > $R/gpurun_out/pmcf_$TAG.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmcw_$TAG -o run --output-format csv -- python3 $B --steps 1 --warmup 0 --eager > $R/gpurun_out/pmcw_$TAG.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmcm_$TAG -o run --output-format csv -- python3 $B --steps 1 --warmup 0 --eager > $R/gpurun_out/pmcm_$TAG.log 2>&1
fi
echo prof-ok

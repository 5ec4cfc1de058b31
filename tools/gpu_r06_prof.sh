#!/bin/bash
# Round-6 profile evidence of the headline step (tiny, B = 32, pitch 3001): rocprofv3 kernel trace + stats of the
# bench command whose line reports the roofline, then separate FETCH_SIZE / WRITE_SIZE and MFMA-busy PMC passes over
# one eager step (each pass its own run, --kernel-trace only beside --pmc).  usage: TAG=r06_p tools/gpu_r06_prof.sh
set -e
R=$GRAFT_REPO_ROOT; T=${TAG:-r06_p}
mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-optimizer --no-dead-block-line --no-refpitch-line --no-fp32-line"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o run --output-format csv -- python3 $B --steps 5 --warmup 2 > $R/gpurun_out/prof_$T.log 2>&1
tail -1 $R/gpurun_out/prof_$T.log | cut -c1-200
P="$B --no-probe --steps 1 --warmup 0"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmcf_$T -o run --output-format csv -- python3 $P > $R/gpurun_out/pmcf_$T.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmcw_$T -o run --output-format csv -- python3 $P > $R/gpurun_out/pmcw_$T.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $R/gpurun_out/pmcm_$T -o run --output-format csv -- python3 $P > $R/gpurun_out/pmcm_$T.log 2>&1
echo prof-ok

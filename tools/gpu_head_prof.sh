#!/bin/bash
# GPU call: the evidence set at HEAD -- rocprofv3 kernel stats of the bench (graph replay, 1 warmup
# + 3 timed = 4 executed steps), FETCH_SIZE and WRITE_SIZE passes over one eager step, and a VALU /
# LDS counter pass over the log-mel microbench.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof3 -o run --output-format csv -- python3 $B --steps 3 --warmup 1 > $R/gpurun_out/prof3.log 2>&1
tail -1 $R/gpurun_out/prof3.log | cut -c1-200
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $B --steps 1 --warmup 0 --eager > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $B --steps 1 --warmup 0 --eager > $R/gpurun_out/pmc_write.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_mel -o run --output-format csv -- python3 $R/tools/microbench.py mel > $R/gpurun_out/pmc_mel.log 2>&1
echo prof-ok

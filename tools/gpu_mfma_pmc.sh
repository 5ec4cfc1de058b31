#!/bin/bash
# One rocprofv3 --pmc pass over one eager bench step: MFMA busy cycles per kernel.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_mfma -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --eager --no-cpu-baseline --no-probe > $R/gpurun_out/pmc_mfma.log 2>&1
echo pmc-ok

#!/bin/bash
# GPU call: one rocprofv3 --pmc pass over a command.  usage: gpu_pmc.sh <outdir> "<counters>" <python args...>
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$1; shift; CTRS=$1; shift
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $R/gpurun_out/$OUT -o run --output-format csv -- python3 "$@" > $R/gpurun_out/$OUT.log 2>&1
echo pmc-ok

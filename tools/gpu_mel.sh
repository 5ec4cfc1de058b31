#!/bin/bash
# GPU call: log-mel parity tests + microbench + kernel stats.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "logmel or golden or mel" > gpurun_out/mel_tests.log 2>&1 || { tail -30 gpurun_out/mel_tests.log; exit 1; }
tail -2 gpurun_out/mel_tests.log
timeout -k 10 120 python tools/microbench.py mel
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mel -o run --output-format csv -- python3 $R/tools/microbench.py mel > $R/gpurun_out/prof_mel.log 2>&1
grep -i "logmel\|Name" $R/gpurun_out/prof_mel/run_kernel_stats.csv | cut -c1-150

#!/bin/bash
# GPU call: a -m gpu test subset (optional), the default bench line, and the headline rocprofv3 profile.
# usage: tools/gpu_evidence.sh TAG ["pytest selection"]
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
TAG=$1
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest $2 -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?; tail -8 gpurun_out/t_$TAG.log; [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-600 gpurun_out/bench_$TAG.json
bash tools/gpu_prof.sh $TAG

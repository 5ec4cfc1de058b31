#!/bin/bash
# round-3 debug: which setting changes the tiny_b2 fp32 gradient scale
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
export TOP=4
for v in "CONC=0 SKIP=0" "CONC=1 SKIP=1" "CONC=0 SKIP=1"; do
  echo "== $v B=2 10s T=64"
  env $v timeout -k 10 200 python -u tools/grad_debug.py 2 10 64 2>&1 | grep -E "^\||replayed|concurrent" || exit 1
done
echo "== B=2 10s T=256"; timeout -k 10 200 python -u tools/grad_debug.py 2 10 256 2>&1 | grep -E "^\||replayed" || exit 1
echo "== B=1 30s T=64"; timeout -k 10 200 python -u tools/grad_debug.py 1 30 64 2>&1 | grep -E "^\||replayed" || exit 1
echo "== B=2 5s T=64"; timeout -k 10 200 python -u tools/grad_debug.py 2 5 64 2>&1 | grep -E "^\||replayed" || exit 1

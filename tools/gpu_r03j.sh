#!/bin/bash
# round-3 debug: per-parameter gradient agreement at tiny_b2 (fp32, decisions replayed) + the fusion tests
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
timeout -k 10 300 python -u tools/grad_debug.py 2 10 64 > $O/grad_debug_b2.log 2>&1 || { tail -20 $O/grad_debug_b2.log; exit 1; }
grep -v Warn $O/grad_debug_b2.log | grep -v detach | head -40
timeout -k 10 300 python -u tools/grad_debug.py 1 10 64 > $O/grad_debug_b1.log 2>&1 || { tail -20 $O/grad_debug_b1.log; exit 1; }
grep -v Warn $O/grad_debug_b1.log | grep -v detach | head -12
timeout -k 10 300 python -u -m pytest tests/test_gpu_fusions.py -v --timeout 120 --timeout-method thread > $O/t_fus.log 2>&1; grep -E "PASSED|FAILED|^E " $O/t_fus.log | head -30

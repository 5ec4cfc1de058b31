#!/bin/bash
# round-3 debug: fp32 parity attention in the model's large-score regime vs float64 and torch fp32
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
timeout -k 10 300 python -u tools/attn_stress.py > $O/attn_stress.log 2>&1 || { tail -20 $O/attn_stress.log; exit 1; }
grep -v Warn $O/attn_stress.log | grep -v amdgpu.ids

#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/blaslt_vs_wide.py 2>&1 | grep -v amdgpu.ids

#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dead_graph_diag.py medium 8 4 eager 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u tools/dead_graph_diag.py medium 8 5 eager steady 2>&1 | grep -v amdgpu.ids || exit 1

#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for m in graph eager eager1; do
timeout -k 10 300 python -u tools/dead_graph_diag.py small 8 5 $m 2>&1 | grep -v amdgpu.ids || exit 1
done
for m in graph eager; do
timeout -k 10 300 python -u tools/dead_graph_diag.py tiny 32 5 $m 2>&1 | grep -v amdgpu.ids || exit 1
done

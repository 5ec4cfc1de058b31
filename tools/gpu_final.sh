#!/bin/bash
# GPU call: the whole -m gpu suite and smoke() at HEAD.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/t_final.log 2>&1 || { tail -30 gpurun_out/t_final.log; exit 1; }
tail -1 gpurun_out/t_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"

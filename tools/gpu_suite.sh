#!/bin/bash
# GPU call: the -m gpu suite (optionally a subset: extra pytest args), logged to gpurun_out/<tag>.log,
# then smoke().  usage: tools/gpu_suite.sh TAG [pytest args...]
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -v -rf --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG.log 2>&1
rc=$?
tail -25 gpurun_out/$TAG.log
[ $rc -le 1 ] || exit $rc   # a timeout / crash: nothing more on the GPU
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"

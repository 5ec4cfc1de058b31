set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in "$@"; do
  if [ $v = prod ]; then timeout -k 10 120 python tools/exp/wr_shapes.py; else ASRX_LIB=$PWD/tools/exp/$v timeout -k 10 120 python tools/exp/wr_shapes.py; fi
done > gpurun_out/wr.log 2>&1
grep -v Warn gpurun_out/wr.log

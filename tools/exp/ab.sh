# usage: bash tools/exp/ab.sh SCRIPT.py prod|libasrx_X.so ...   (A/B timing of library variants)
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
S=$1; shift
for v in "$@"; do
  if [ $v = prod ]; then timeout -k 10 150 python $S; else ASRX_LIB=$PWD/tools/exp/$v timeout -k 10 150 python $S; fi
done > gpurun_out/ab.log 2>&1
grep -v -e Warn -e amdgpu.ids gpurun_out/ab.log

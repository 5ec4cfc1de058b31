cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export GEMM_SHAPES="8192,384,384;8192,256,384;8192,384,256;49152,64,64;8192,384,1152" GEMM_NJ=1 GEMM_ITERS=100
for v in prod libasrx_nofast.so prod libasrx_nofast.so; do
  echo "== $v"
  if [ $v = prod ]; then timeout -k 10 150 python tools/gemm_micro.py; else ASRX_LIB=$PWD/tools/exp/$v timeout -k 10 150 python tools/gemm_micro.py; fi
done > gpurun_out/nj1_ab.log 2>&1
grep -E "==|nj1" gpurun_out/nj1_ab.log

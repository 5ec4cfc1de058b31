cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export GEMM_SHAPES="192064,384,384;192064,1536,384;192064,384,1536;96000,384,384" GEMM_NJ=3 GEMM_ITERS=20 GEMM_BIAS=1
for v in prod libasrx_epidirect.so prod libasrx_epidirect.so; do
  echo "== $v"
  if [ $v = prod ]; then timeout -k 10 150 python tools/gemm_micro.py; else ASRX_LIB=$PWD/tools/exp/$v timeout -k 10 150 python tools/gemm_micro.py; fi
done > gpurun_out/epidirect_ab.log 2>&1
grep -E "==|nj3" gpurun_out/epidirect_ab.log

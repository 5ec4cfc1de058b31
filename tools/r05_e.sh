set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export GEMM_SHAPES="192064,384,384;192064,1536,384;192064,384,1536;8192,384,384" GEMM_NJ=3 GEMM_ITERS=20 GEMM_ABF=1 GEMM_VARIANT=1
for v in p2base p2slow p2abl1 p2abl2 p2abl4 p2abl8 p2abl9 p2base; do
  echo "== $v"; ASRX_LIB=$PWD/tools/exp/libasrx_$v.so timeout -k 10 120 python tools/gemm_micro.py
done > gpurun_out/r05_p2_ablation.log 2>&1
grep -E "==|nj" gpurun_out/r05_p2_ablation.log

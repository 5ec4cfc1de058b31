set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export GEMM_SHAPES="192064,384,384;192064,384,1536;192064,1536,384" GEMM_NJ=3 GEMM_ITERS=20 GEMM_ABF=1 GEMM_VARIANT=1
for c in 0 1; do
for v in base p2abl1 p2abl2 p2abl4 p2abl8 p2abl6 p2abl12 base; do
  if [ $v = base ]; then L=$PWD/asr-model_amd/asrx/libasrx.so; else L=$PWD/tools/exp/libasrx_$v.so; fi
  echo "== $v cbf=$c"; GEMM_CBF=$([ $c = 1 ] && echo 1 || echo "") ASRX_LIB=$L timeout -k 10 120 python tools/gemm_micro.py
done
done > gpurun_out/r05_p2_ablation.log 2>&1
grep -E "==|nj" gpurun_out/r05_p2_ablation.log

set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_ws.py -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/r05_t_tests.log 2>&1 || { tail -30 gpurun_out/r05_t_tests.log; exit 1; }
tail -2 gpurun_out/r05_t_tests.log
export GEMM_SHAPES="192064,384,384;192064,1536,384;192064,1152,384;192064,768,384;96000,384,384" GEMM_NJ=3 GEMM_ITERS=20
for c in 0 1; do for v in ws3 ws64 p2 ws3; do
  case $v in ws3) L=$PWD/asr-model_amd/asrx/libasrx.so; V=13;; p2) L=$PWD/asr-model_amd/asrx/libasrx.so; V=1;; *) L=$PWD/tools/exp/libasrx_$v.so; V=13;; esac
  echo "== $v cbf=$c"; GEMM_CBF=$([ $c = 1 ] && echo 1 || echo "") ASRX_LIB=$L GEMM_VARIANT=$V timeout -k 10 120 python tools/gemm_micro.py
done; done > gpurun_out/r05_ws_micro3.log 2>&1
grep -E "==|nj" gpurun_out/r05_ws_micro3.log

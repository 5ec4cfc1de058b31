set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_ws.py tests/test_gpu_gemm_p2.py tests/test_gpu_rot_fused.py -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/r05_q_tests.log 2>&1 || { tail -30 gpurun_out/r05_q_tests.log; exit 1; }
tail -2 gpurun_out/r05_q_tests.log
export GEMM_SHAPES="192064,384,384;192064,1536,384;192064,1152,384;192064,768,384;192064,256,384;96000,384,384" GEMM_NJ=3 GEMM_ITERS=20
for c in 0 1; do for v in 5 1 5 1; do
  echo "== variant $v cbf=$c"; GEMM_CBF=$([ $c = 1 ] && echo 1 || echo "") GEMM_VARIANT=$v timeout -k 10 120 python tools/gemm_micro.py
done; done > gpurun_out/r05_ws_micro.log 2>&1
grep -E "==|nj" gpurun_out/r05_ws_micro.log
B="--no-cpu-baseline --no-dead-block-line --no-refpitch-line --no-optimizer"
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $B > gpurun_out/r05_q_bench.json 2>gpurun_out/r05_q_bench.err
cut -c1-400 gpurun_out/r05_q_bench.json

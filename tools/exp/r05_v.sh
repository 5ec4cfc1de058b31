#!/bin/bash
# Epilogue batching A/B: beta = 0 / 1 and the residual GEMM, old library (inline reads) vs new (batched reads).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/r05_v.txt
: > $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_ws.py tests/test_gpu_gemm_p2.py tests/test_gpu_gemm_mel.py tests/test_gpu_gemm_x3.py > gpurun_out/r05_v_tests.log 2>&1 || { tail -30 gpurun_out/r05_v_tests.log; exit 1; }
tail -3 gpurun_out/r05_v_tests.log
S="192064,384,384;96032,384,384;192064,384,1536;192064,1536,384"
for lib in tools/exp/libasrx_epi_old.so asr-model_amd/asrx/libasrx.so; do
  for beta in 0 1; do
    echo "== $lib beta=$beta" >> $O
    ASRX_LIB=$lib GEMM_BETA=$beta GEMM_SHAPES="$S" GEMM_NJ=1,3 GEMM_ITERS=30 timeout -k 10 240 python -u tools/gemm_micro.py >> $O 2>&1 || exit 1
  done
done
cat $O

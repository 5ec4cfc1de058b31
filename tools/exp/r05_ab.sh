#!/bin/bash
# Row-kernel instruction cuts (AbbyNormal forward zero pads + float2 halo, paired DPP reductions): micro A/B with
# checksums, HEAD library vs the working tree, arms interleaved on one box; then the row-kernel GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/r05_ab_micro.txt
: > $O
for lib in tools/exp/libasrx_head.so asr-model_amd/asrx/libasrx.so tools/exp/libasrx_head.so asr-model_amd/asrx/libasrx.so; do
  echo "== $lib" >> $O
  ASRX_LIB=$lib timeout -k 10 300 python -u tools/microbench.py abby msrow >> $O 2>&1 || exit 1
done
cat $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fusions.py tests/test_gpu_ops.py tests/test_gpu_bf16_storage.py tests/test_gpu_model.py > gpurun_out/r05_ab_tests.log 2>&1 || { tail -30 gpurun_out/r05_ab_tests.log; exit 1; }
tail -3 gpurun_out/r05_ab_tests.log

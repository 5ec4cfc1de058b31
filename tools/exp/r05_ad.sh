#!/bin/bash
# wgrad_wr_kernel<bf16 dY, bf16 X> with 4 k-steps of loads in flight (default) vs 2 (tools/exp/libasrx_d2.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/r05_ad_micro.txt
: > $O
for lib in asr-model_amd/asrx/libasrx.so tools/exp/libasrx_d2.so asr-model_amd/asrx/libasrx.so tools/exp/libasrx_d2.so; do
ASRX_LIB=$lib timeout -k 10 300 python -u - >> $O 2>&1 <<'PY' || exit 1
import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "asr-model_amd"), os.path.join(os.getcwd(), "tools")]
import torch
from microbench import timeit
from asrx import lib
dev = torch.device("cuda:0")
for (M, N, R) in [(1536, 384, 192064), (384, 384, 192064), (1536, 384, 96000), (40000, 384, 8192)]:
    dy = torch.randn(R, M, device=dev).to(torch.bfloat16); xb = torch.randn(R, N, device=dev).to(torch.bfloat16)
    out = torch.zeros(M, N, device=dev)
    sk = max(1, min(512 // (((M + 127) // 128) * ((N + 127) // 128)), R // 256))
    f = lambda: lib.call("asrx_wgrad_bf16_ab", lib.ptr(dy), M, lib.ptr(xb), 1, N, lib.ptr(out), N, M, N, R, sk, lib.stream())
    t = timeit(f, iters=20)
    print(f"{os.environ['ASRX_LIB'][-14:]} wgrad bf16/bf16 M={M} N={N} R={R}: {t*1e6:8.1f} us {2*M*N*R/t/1e12:6.1f} TF/s ck {float(out.double().sum()):.6e}", flush=True)
PY
done
cat $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ce_fused.py tests/test_gpu_fusions.py > gpurun_out/r05_ad_tests.log 2>&1 || { tail -30 gpurun_out/r05_ad_tests.log; exit 1; }
tail -2 gpurun_out/r05_ad_tests.log

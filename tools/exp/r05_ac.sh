#!/bin/bash
# Wide weight-gradient items: tests, then micro (variant 1 vs 0) at the step's bf16-X shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wgrad_w3.py tests/test_gpu_fusions.py tests/test_gpu_bf16_storage.py > gpurun_out/r05_ac_tests.log 2>&1 || { tail -40 gpurun_out/r05_ac_tests.log; exit 1; }
tail -2 gpurun_out/r05_ac_tests.log
timeout -k 10 300 python -u - > gpurun_out/r05_ac_micro.txt 2>&1 <<'PY' || { cat gpurun_out/r05_ac_micro.txt; exit 1; }
import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "asr-model_amd"), os.path.join(os.getcwd(), "tools")]
import torch
from microbench import timeit
from asrx import lib
dev = torch.device("cuda:0")
for rep in range(2):
    for v in (1, 0):
        lib.load().asrx_set_wgrad_variant(v)
        for (M, N, R) in [(384, 384, 192064), (384, 384, 96000), (1536, 384, 192064), (384, 1536, 192064), (384, 384, 8192)]:
            dy = torch.randn(R, M, device=dev); xb = torch.randn(R, N, device=dev).to(torch.bfloat16)
            out = torch.zeros(M, N, device=dev); db = torch.zeros(M, device=dev)
            sk = max(1, min(512 // (((M + 127) // 128) * ((N + 127) // 128)), R // 256))
            f = lambda: lib.call("asrx_wgrad_bias", lib.ptr(dy), 0, M, lib.ptr(xb), 1, N, lib.ptr(out), N, lib.ptr(db), M, N, R, sk, lib.stream())
            t = timeit(f, iters=20)
            print(f"variant {v} wgrad M={M} N={N} R={R}: {t*1e6:8.1f} us {2*M*N*R/t/1e12:6.1f} TF/s {R*(4*M+2*N)/t/1e9:6.0f} GB/s", flush=True)
            del dy, xb
PY
cat gpurun_out/r05_ac_micro.txt

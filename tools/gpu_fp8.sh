set -e; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread -k "attention" > gpurun_out/f8_tests.log 2>&1 || { tail -40 gpurun_out/f8_tests.log; exit 1; }
tail -3 gpurun_out/f8_tests.log
timeout -k 10 200 python tools/microbench.py attn > gpurun_out/attn_mb.log 2>&1; grep -v Warn gpurun_out/attn_mb.log
timeout -k 10 200 python tools/decode_bench.py small 8 32 bf16 > gpurun_out/dec_small_bf16.json 2>gpurun_out/dec.err; cat gpurun_out/dec_small_bf16.json
timeout -k 10 200 python tools/decode_bench.py small 8 32 fp8 > gpurun_out/dec_small_fp8.json 2>>gpurun_out/dec.err; cat gpurun_out/dec_small_fp8.json

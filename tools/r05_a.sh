set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_p2.py > gpurun_out/r05_p2_tests.log 2>&1 || { tail -30 gpurun_out/r05_p2_tests.log; exit 1; }
tail -2 gpurun_out/r05_p2_tests.log
export GEMM_SHAPES="192064,384,384;192064,1536,384;192064,384,1536;192064,1152,384;96000,384,384;8192,384,384;8192,1536,384" GEMM_NJ=3 GEMM_ITERS=20
for v in 1 0 1 0; do echo "== variant $v"; GEMM_VARIANT=$v timeout -k 10 200 python tools/gemm_micro.py; done > gpurun_out/r05_p2_micro.log 2>&1
grep -E "==|nj" gpurun_out/r05_p2_micro.log
unset GEMM_SHAPES GEMM_NJ GEMM_ITERS
timeout -k 10 200 python tools/attn_micro.py > gpurun_out/r05_attn_micro.log 2>&1
grep variant gpurun_out/r05_attn_micro.log
timeout -k 10 300 python3 -u tools/gemm_table.py tiny 32 > gpurun_out/r05_gemm_table_v1.txt 2>&1
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dead-block-line --no-refpitch-line > gpurun_out/r05_bench_v1.json 2> gpurun_out/r05_bench_v1.err
tail -c 600 gpurun_out/r05_bench_v1.json
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dead-block-line --no-refpitch-line --eager --no-probe > gpurun_out/r05_bench_eager.json 2> gpurun_out/r05_bench_eager.err
timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --precision fp32 --no-cpu-baseline --no-dead-block-line --no-refpitch-line > gpurun_out/r05_bench_fp32.json 2> gpurun_out/r05_bench_fp32.err
echo done

set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_gemm_x3.py > gpurun_out/r05_d_x3gemm.log 2>&1 || { tail -30 gpurun_out/r05_d_x3gemm.log; exit 1; }
grep -E "passed|failed" gpurun_out/r05_d_x3gemm.log | tail -1
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread tests/test_gpu_model_configs.py -k "x3" > gpurun_out/r05_d_x3parity.log 2>&1 || { tail -40 gpurun_out/r05_d_x3parity.log; exit 1; }
grep -E "x3 \{|passed|failed" gpurun_out/r05_d_x3parity.log | cut -c1-400
timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --precision x3 --no-cpu-baseline --no-dead-block-line --no-refpitch-line --no-optimizer > gpurun_out/r05_bench_x3.json 2> gpurun_out/r05_bench_x3.err
tail -c 900 gpurun_out/r05_bench_x3.json
echo done

# round-3 GPU check, stage B: identity checks, bf16-storage tests, then the core suites and the bench
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 100 python tools/debug_ln.py > gpurun_out/dbg_ln.log 2>&1; tail -2 gpurun_out/dbg_ln.log
timeout -k 10 100 python tools/debug_storage2.py > gpurun_out/dbg3.log 2>&1; grep all_on gpurun_out/dbg3.log
FILES="tests/test_gpu_bf16_storage.py tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_gemm_mel.py tests/test_gpu_model_configs.py tests/test_gpu_dist.py tests/test_gpu_generate.py tests/test_gpu_optim.py tests/test_gpu_data.py tests/test_gpu_pitch.py"
rc=0
timeout -k 10 1000 python -u -m pytest $FILES -v --timeout 300 --timeout-method thread > gpurun_out/t_r03.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|Fatal" gpurun_out/t_r03.log | head -30
# a crash (abort / segfault / time limit) may have left the GPU faulted: start nothing more on it
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
grep -E "passed|failed" gpurun_out/t_r03.log | tail -2
timeout -k 10 400 python bench.py > gpurun_out/bench_r03.json 2> gpurun_out/bench_r03.err || { tail -30 gpurun_out/bench_r03.err; exit 1; }
cat gpurun_out/bench_r03.json

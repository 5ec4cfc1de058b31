set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_p2.py > gpurun_out/r05_p2_tests.log 2>&1 || { tail -30 gpurun_out/r05_p2_tests.log; exit 1; }
tail -3 gpurun_out/r05_p2_tests.log
export GEMM_SHAPES="192064,384,384;192064,1536,384;192064,384,1536;192064,1152,384;96000,384,384;8192,384,384;8192,1536,384" GEMM_NJ=3 GEMM_ITERS=20
for v in 1 0 1 0; do echo "== variant $v"; GEMM_VARIANT=$v timeout -k 10 200 python tools/gemm_micro.py; done > gpurun_out/r05_p2_micro.log 2>&1
grep -E "==|nj" gpurun_out/r05_p2_micro.log

set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_p2.py tests/test_gpu_ops.py -k 'p2 or attention or attn' > gpurun_out/r05_c_tests.log 2>&1 || { tail -30 gpurun_out/r05_c_tests.log; exit 1; }
tail -1 gpurun_out/r05_c_tests.log
export GEMM_SHAPES="8192,384,384;8192,1536,384;8192,384,1536;8192,1152,384;8192,256,384" GEMM_NJ=1 GEMM_ITERS=30
for v in 2 0 2 0; do echo "== variant $v"; GEMM_VARIANT=$v timeout -k 10 200 python tools/gemm_micro.py; done > gpurun_out/r05_nj1_micro.log 2>&1
grep -E "==|nj" gpurun_out/r05_nj1_micro.log
unset GEMM_SHAPES GEMM_NJ GEMM_ITERS
timeout -k 10 300 python tools/attn_micro.py 2 > gpurun_out/r05_attn_micro_v2.log 2>&1
grep rep gpurun_out/r05_attn_micro_v2.log
B="--no-cpu-baseline --no-dead-block-line --no-refpitch-line --no-probe --no-optimizer"
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $B > gpurun_out/r05_c_graph$i.json 2>/dev/null
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $B --eager > gpurun_out/r05_c_eager$i.json 2>/dev/null
python3 -c "
import json
for f in ['gpurun_out/r05_c_graph$i.json','gpurun_out/r05_c_eager$i.json']:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['launch'])
"
done
echo done

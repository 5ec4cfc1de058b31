set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/gemm_table.py tiny 32 > gpurun_out/r05_g_gemm_table.txt 2>&1
B="--no-cpu-baseline --no-dead-block-line --no-refpitch-line --no-probe --no-optimizer"
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $B > gpurun_out/r05_g_graph$i.json 2>/dev/null
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $B --eager > gpurun_out/r05_g_eager$i.json 2>/dev/null
done
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $B --dist-single > gpurun_out/r05_g_distsingle.json 2>gpurun_out/r05_g_distsingle.err
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/r05_g_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['launch'])
"

set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B="--no-cpu-baseline --no-dead-block-line --no-refpitch-line --no-probe --no-optimizer"
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $B > gpurun_out/r05_m_tiny_eager.json 2>/dev/null
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $B --graph > gpurun_out/r05_m_tiny_graph.json 2>/dev/null
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 $B --config small --batch 8 > gpurun_out/r05_m_small_eager.json 2>/dev/null
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 $B --config small --batch 8 --graph > gpurun_out/r05_m_small_graph.json 2>/dev/null
timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 $B --config medium --batch 8 --graph > gpurun_out/r05_m_medium8_graph.json 2>gpurun_out/r05_m_medium8_graph.err || tail -3 gpurun_out/r05_m_medium8_graph.err
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/r05_m_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['host_issue_ms_per_step'], d['launch'])
"

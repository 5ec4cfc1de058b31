set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B="--no-cpu-baseline --no-dead-block-line --no-refpitch-line --no-probe --no-optimizer"
for b in 32 16 8; do
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $B --batch $b > gpurun_out/r05_o_b$b.json 2>gpurun_out/r05_o_b$b.err
done
ASRX_CTYPES=1 timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $B > gpurun_out/r05_o_b32_ctypes.json 2>/dev/null
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/r05_o_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['host_issue_ms_per_step'], d['launch'])
"
timeout -k 10 240 python3 tools/host_prof.py tiny 32 5 > gpurun_out/r05_hostprof2.txt 2>&1
head -3 gpurun_out/r05_hostprof2.txt
timeout -k 10 120 python3 tools/launch_cost.py 500 > gpurun_out/r05_launch_cost.txt 2>&1
cat gpurun_out/r05_launch_cost.txt

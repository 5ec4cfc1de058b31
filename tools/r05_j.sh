set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B="--no-cpu-baseline --no-dead-block-line --no-refpitch-line --no-probe --no-optimizer"
for i in 1 2; do for d in start mid end; do
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $B --dead-at $d > gpurun_out/r05_j_$d$i.json 2>gpurun_out/r05_j_$d$i.err
done; done
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/r05_j_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['launch'])
"
timeout -k 10 600 python3 -u bench.py --config medium --batch 8 --steps 3 --warmup 1 $B > gpurun_out/r05_j_medium8.json 2>gpurun_out/r05_j_medium8.err || tail -5 gpurun_out/r05_j_medium8.err
tail -c 400 gpurun_out/r05_j_medium8.json

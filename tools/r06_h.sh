#!/bin/bash
# round 6, call h: parity configs with the metrics collector, the default bench line (fp32 side line), the 2-rank
# rehearsal (pinning, bf16 wire), --dist-single at small and medium
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export ASRX_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/r06_parity_metrics.jsonl
rm -f $ASRX_PARITY_LOG
timeout -k 10 900 python -u -m pytest tests/test_gpu_model_configs.py -m gpu -v -rf --timeout 400 --timeout-method thread > gpurun_out/r06_h_configs.log 2>&1
rc=$?; tail -5 gpurun_out/r06_h_configs.log; [ $rc -le 1 ] || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r06_h_tiny.json 2> gpurun_out/r06_h_tiny.err || { tail -20 gpurun_out/r06_h_tiny.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r06_h_tiny.json')); print(d['value'], d.get('fp32_workload'))"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --batch 4 --dist-backend gloo --same-device --bf16-grads > gpurun_out/r06_h_rehearsal.log 2>&1 || { tail -20 gpurun_out/r06_h_rehearsal.log; exit 1; }
tail -1 gpurun_out/r06_h_rehearsal.log | cut -c1-200; grep -o '"cpu_affinity_by_rank[^]]*]' gpurun_out/r06_h_rehearsal.log
B="--no-cpu-baseline --no-refpitch-line --no-dead-block-line --no-optimizer --no-fp32-line --dist-single"
timeout -k 10 400 python -u bench.py $B --config small --batch 8 > gpurun_out/r06_h_small_distsingle.json 2> gpurun_out/r06_h_small_ds.err || { tail -20 gpurun_out/r06_h_small_ds.err; exit 1; }
timeout -k 10 400 python -u bench.py $B --config medium --batch 8 --steps 3 > gpurun_out/r06_h_medium_distsingle.json 2> gpurun_out/r06_h_medium_ds.err || { tail -20 gpurun_out/r06_h_medium_ds.err; exit 1; }
for f in small medium; do cut -c1-200 gpurun_out/r06_h_${f}_distsingle.json; done

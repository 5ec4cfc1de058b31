#!/bin/bash
# One-GPU rehearsal of the N>1 bench path: 2 ranks on cuda:0 over gloo (GradSync hooks, comm
# stream, bucket all-reduce, max-over-ranks timing).  RCCL itself needs one GPU per rank.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --batch 4 --dist-backend gloo --same-device > gpurun_out/dist_rehearsal.log 2>&1
tail -3 gpurun_out/dist_rehearsal.log

#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=r06_ctrl4 bash tools/gpu_r06.sh suite || exit 1
timeout -k 10 400 python -u bench.py --config small --batch 8 --steps 6 --warmup 2 --no-fp32-line --no-cpu-baseline --no-refpitch-line --no-dead-block-line --no-probe > gpurun_out/r06_small_ctrl4.json 2>gpurun_out/r06_small_ctrl4.err || exit 1
cut -c1-300 gpurun_out/r06_small_ctrl4.json

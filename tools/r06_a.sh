#!/bin/bash
# round 6, call a: dead-block graph tests + rotary variant tests, then tiny / small / medium bench lines
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=r06_a
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_rot_fused.py tests/test_gpu_small_linear.py -m gpu -v -rf -s --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -15 gpurun_out/${T}_tests.log; [ $rc -le 1 ] || exit $rc
B="--no-cpu-baseline --no-refpitch-line --no-dead-block-line --no-optimizer"
timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_tiny.json 2> gpurun_out/${T}_tiny.err || { tail -20 gpurun_out/${T}_tiny.err; exit 1; }
cut -c1-400 gpurun_out/${T}_tiny.json
timeout -k 10 300 python -u bench.py $B --config small --batch 8 > gpurun_out/${T}_small.json 2> gpurun_out/${T}_small.err || { tail -20 gpurun_out/${T}_small.err; exit 1; }
cut -c1-400 gpurun_out/${T}_small.json
timeout -k 10 400 python -u bench.py $B --config medium --batch 8 --steps 3 > gpurun_out/${T}_medium.json 2> gpurun_out/${T}_medium.err || { tail -20 gpurun_out/${T}_medium.err; exit 1; }
cut -c1-400 gpurun_out/${T}_medium.json

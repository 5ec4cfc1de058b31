#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lt_census.py small 8 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u tools/lt_census.py tiny 32 2>&1 | grep -v amdgpu.ids || exit 1
B="--no-cpu-baseline --no-refpitch-line --no-dead-block-line --no-optimizer --no-fp32-line --no-probe"
for v in 0 1 0 1; do
ASRX_LIBRARY_GEMM=$v timeout -k 10 300 python -u bench.py $B --config small --batch 8 > gpurun_out/r06_o_small_$v.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r06_o_small_$v.json')); print('small lib=$v', d['value'], d['ms_per_step'])"
done

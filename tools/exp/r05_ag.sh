#!/bin/bash
# nj = 1 launches on gemm_p2 (variant 6 = 2 + 4) vs the default (5), interleaved, headline config
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
A="--no-cpu-baseline --no-refpitch-line --no-dead-block-line"
for v in 5 6 5 6; do
  GEMM_VARIANT=$v timeout -k 10 400 python -u tools/exp/bench_variant.py $A > gpurun_out/r05_ag_$v.json 2> gpurun_out/r05_ag_$v.err || { tail -20 gpurun_out/r05_ag_$v.err; exit 1; }
  echo "variant $v: $(cut -c1-170 gpurun_out/r05_ag_$v.json | grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": 5, "warmup": 2, "ms_per_step": [0-9.]*')"
done

#!/bin/bash
# seg_reduce (per-sample chunk sums) with batched loads: tests, step kernel trace (8.7 us per launch before), bench line
# step's kernel trace (msheath_ctrl_fwd 11.4 us, msheath_ctrl_bwd 20.7 us before) and a bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_bf16_storage.py tests/test_gpu_model_configs.py > gpurun_out/r05_ai_tests.log 2>&1 || { tail -30 gpurun_out/r05_ai_tests.log; exit 1; }
tail -1 gpurun_out/r05_ai_tests.log
bash tools/gpu_prof.sh r05_ai
python3 tools/replay_step.py gpurun_out/prof_r05_ai/run_kernel_trace.csv r05_ai > gpurun_out/r05_ai_step.txt
grep -h "seg_reduce\|msheath_ctrl" gpurun_out/r05_ai_step.txt | cut -c1-90
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-refpitch-line --no-dead-block-line > gpurun_out/r05_ai_bench.json 2> gpurun_out/r05_ai_bench.err || { tail -20 gpurun_out/r05_ai_bench.err; exit 1; }
cut -c1-200 gpurun_out/r05_ai_bench.json

#!/bin/bash
# row_normalize_bwd with one load round trip per row (9.8 us per launch before): tests, step trace, bench line
# step's kernel trace (msheath_ctrl_fwd 11.4 us, msheath_ctrl_bwd 20.7 us before) and a bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_bf16_storage.py tests/test_gpu_model_configs.py > gpurun_out/r05_aj_tests.log 2>&1 || { tail -30 gpurun_out/r05_aj_tests.log; exit 1; }
tail -1 gpurun_out/r05_aj_tests.log
bash tools/gpu_prof.sh r05_aj
python3 tools/replay_step.py gpurun_out/prof_r05_aj/run_kernel_trace.csv r05_aj > gpurun_out/r05_aj_step.txt
grep -h "row_normalize_bwd" gpurun_out/r05_aj_step.txt | cut -c1-90
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-refpitch-line --no-dead-block-line > gpurun_out/r05_aj_bench.json 2> gpurun_out/r05_aj_bench.err || { tail -20 gpurun_out/r05_aj_bench.err; exit 1; }
cut -c1-200 gpurun_out/r05_aj_bench.json

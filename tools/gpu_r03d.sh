#!/bin/bash
# round-3: parity metrics with decision replay, the re-gated op tests, then the rocprof evidence passes
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py::test_abby_normal tests/test_gpu_bf16_storage.py -v -s --timeout 120 --timeout-method thread > gpurun_out/t_r03d.log 2>&1; rc=$?
grep -E "PASSED|FAILED|worst" gpurun_out/t_r03d.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u tools/parity_measure.py > gpurun_out/parity_r03.jsonl 2> gpurun_out/parity_r03.err || { tail -20 gpurun_out/parity_r03.err; exit 1; }
bash tools/gpu_prof_r03.sh r03a

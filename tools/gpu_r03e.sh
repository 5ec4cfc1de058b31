#!/bin/bash
# round-3: fused CE tests, bf16-storage gradient bisect, then parity metrics with mode-2 cond decisions
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ce_fused.py -v -x --timeout 120 --timeout-method thread > gpurun_out/t_ce.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|assert" gpurun_out/t_ce.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/debug_storage_grad.py > gpurun_out/dbg_sgrad.log 2>&1 || { tail -20 gpurun_out/dbg_sgrad.log; exit 1; }
cat gpurun_out/dbg_sgrad.log
timeout -k 10 600 python -u tools/parity_measure.py $PCASES > gpurun_out/parity_r03b.jsonl 2> gpurun_out/parity_r03b.err || { tail -20 gpurun_out/parity_r03b.err; exit 1; }
echo parity-ok

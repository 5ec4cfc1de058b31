#!/bin/bash
# round-3 final: fused-bias whole-model test and smoke(), then the final evidence (PMC passes, small / medium)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
timeout -k 10 300 python -u -m pytest tests/test_gpu_fusions.py -m gpu -q -k "model_bias" --timeout 200 --timeout-method thread > $O/t_r03y.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|^E " $O/t_r03y.log | head -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r03y.log 2>&1 || { tail -5 $O/smoke_r03y.log; exit 1; }
tail -1 $O/smoke_r03y.log
bash $S/tools/gpu_r03v.sh

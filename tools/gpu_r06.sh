#!/bin/bash
# Round-6 GPU evidence: the whole -m gpu suite (parity metrics collected into gpurun_out/${TAG}_parity.jsonl),
# smoke(), then the default bench line.  usage: TAG=r06_x tools/gpu_r06.sh [suite|bench|all]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r06}
what=${1:-all}
if [ $what = suite ] || [ $what = all ]; then
  export ASRX_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/${T}_parity.jsonl
  rm -f $ASRX_PARITY_LOG
  timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rf --timeout 400 --timeout-method thread > gpurun_out/${T}_suite.log 2>&1
  rc=$?; tail -4 gpurun_out/${T}_suite.log; grep -E "FAILED|ERROR" gpurun_out/${T}_suite.log | head -20
  [ $rc -le 1 ] || exit $rc
  unset ASRX_PARITY_LOG
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
  tail -2 gpurun_out/${T}_smoke.log
fi
if [ $what = bench ] || [ $what = all ]; then
  timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['ms_per_step'], {k: d[k].get('value') for k in ('fp32_workload','x3_workload','dead_block_eliminated','refpitch_workload') if k in d}, d.get('cpu_baseline',{}).get('value'))"
fi

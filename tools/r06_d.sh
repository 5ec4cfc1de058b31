#!/bin/bash
# round 6, call d: composite MSheath forward parity, model tests, then tiny / small / medium bench lines
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r06_d}
[ -n "$SKIPTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_msheath_composite.py tests/test_gpu_model.py tests/test_gpu_generate.py -m gpu -v -rf -s --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/${T}_tests.log | tail -30; [ $rc -eq 0 ] || exit 1
B="--no-cpu-baseline --no-refpitch-line --no-dead-block-line --no-optimizer"
for c in "tiny --batch 32" "small --batch 8" "medium --batch 8 --steps 3"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -k 10 400 python -u bench.py $B --config $c > gpurun_out/${T}_$n.json 2> gpurun_out/${T}_$n.err || { tail -20 gpurun_out/${T}_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_$n.json')); print('$n', d['value'], d['ms_per_step'], d['host_issue_ms_per_step'], d.get('host_issue_from_idle_ms'), d.get('step_from_idle_ms'))"
done

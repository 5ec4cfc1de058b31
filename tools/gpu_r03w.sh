#!/bin/bash
# round-3: the GPU suite from the model-config tests on (the previous call stopped there), the fusion tests,
# then the bench line + kernel trace
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
rc=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_fusions.py tests/test_gpu_model_configs.py tests/test_gpu_ops.py tests/test_gpu_optim.py tests/test_gpu_pitch.py -m gpu -q --timeout 300 --timeout-method thread > $O/t_r03w.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|Fatal|passed|failed" $O/t_r03w.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
BA="$S/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03w -o run --output-format csv -- python3 $BA --steps 3 --warmup 1 > $O/prof_r03w.log 2>&1 || { tail -5 $O/prof_r03w.log; exit 1; }
cd $S && timeout -k 10 400 python bench.py > $O/bench_r03w.json 2> $O/bench_r03w.err || { tail -30 $O/bench_r03w.err; exit 1; }
cat $O/bench_r03w.json

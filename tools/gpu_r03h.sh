#!/bin/bash
# round-3: the whole -m gpu suite, then rocprof kernel trace of the bench and the bench line
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R/.snap 2>/dev/null || cd $R
rc=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/t_r03h.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|Fatal" $O/t_r03h.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
grep -E "passed|failed" $O/t_r03h.log | tail -2
cd /tmp && export TMPDIR=/tmp
S=$R/.snap; [ -d $S ] || S=$R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03h -o run --output-format csv -- python3 $S/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line --steps 3 --warmup 1 > $O/prof_r03h.log 2>&1 || { tail -5 $O/prof_r03h.log; exit 1; }
tail -1 $O/prof_r03h.log | cut -c1-300
cd $S && timeout -k 10 400 python bench.py > $O/bench_r03h.json 2> $O/bench_r03h.err || { tail -30 $O/bench_r03h.err; exit 1; }
cat $O/bench_r03h.json

#!/bin/bash
# round-3 evidence A: the whole -m gpu suite, rocprof kernel trace + stats of the bench, PMC FETCH /
# WRITE / MFMA-busy passes over one eager step, and the default bench line
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
rc=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/t_r03m.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|Fatal" $O/t_r03m.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
grep -E "passed|failed" $O/t_r03m.log | tail -2
cd /tmp && export TMPDIR=/tmp
BA="$S/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03m -o run --output-format csv -- python3 $BA --steps 3 --warmup 1 > $O/prof_r03m.log 2>&1 || { tail -5 $O/prof_r03m.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmcf_r03m -o run --output-format csv -- python3 $BA --steps 1 --warmup 0 --eager > $O/pmcf_r03m.log 2>&1 || { tail -5 $O/pmcf_r03m.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmcw_r03m -o run --output-format csv -- python3 $BA --steps 1 --warmup 0 --eager > $O/pmcw_r03m.log 2>&1 || { tail -5 $O/pmcw_r03m.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $O/pmcm_r03m -o run --output-format csv -- python3 $BA --steps 1 --warmup 0 --eager > $O/pmcm_r03m.log 2>&1 || { tail -5 $O/pmcm_r03m.log; exit 1; }
cd $S && timeout -k 10 400 python bench.py > $O/bench_r03m.json 2> $O/bench_r03m.err || { tail -30 $O/bench_r03m.err; exit 1; }
cat $O/bench_r03m.json

#!/bin/bash
# round-3: launch census by call site, PMC FETCH / WRITE passes over one eager step (traffic table v2)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
timeout -k 10 300 python -u tools/call_census.py tiny 32 > $O/census_r03r.txt 2>&1 || { tail -5 $O/census_r03r.txt; exit 1; }
head -45 $O/census_r03r.txt
cd /tmp && export TMPDIR=/tmp
BA="$S/bench.py --no-cpu-baseline --no-probe --no-optimizer --no-dead-block-line --no-refpitch-line"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmcf_r03r -o run --output-format csv -- python3 $BA --steps 1 --warmup 0 --eager > $O/pmcf_r03r.log 2>&1 || { tail -5 $O/pmcf_r03r.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmcw_r03r -o run --output-format csv -- python3 $BA --steps 1 --warmup 0 --eager > $O/pmcw_r03r.log 2>&1 || { tail -5 $O/pmcw_r03r.log; exit 1; }
echo pmc-ok

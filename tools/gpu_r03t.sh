#!/bin/bash
# round-3: launch census with callers (colsum / lincomb origins)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
S=$R/.snap; [ -d $S ] || S=$R
cd $S
timeout -k 10 300 python -u tools/call_census.py tiny 32 > $O/census_r03t.txt 2>&1 || { tail -5 $O/census_r03t.txt; exit 1; }
grep -E "colsum|lincomb|act_bwd|act_fwd|zero" $O/census_r03t.txt | head -40

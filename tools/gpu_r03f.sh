#!/bin/bash
# round-3: bf16-storage gradient bisect by site, and the per-shape GEMM table of one eager step
# (runs the frozen copy .snap/ when present; outputs go to the top-level gpurun_out/)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R/.snap 2>/dev/null || cd $R
timeout -k 10 300 python -u tools/debug_storage_grad.py > $O/dbg_sgrad2.log 2>&1 || { tail -20 $O/dbg_sgrad2.log; exit 1; }
grep -v Warn $O/dbg_sgrad2.log | grep -v detach
timeout -k 10 300 python -u tools/gemm_table.py > $O/gemm_table_r03.txt 2>&1 || { tail -20 $O/gemm_table_r03.txt; exit 1; }
head -60 $O/gemm_table_r03.txt

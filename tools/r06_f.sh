#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/host_prof.py medium 8 2 > gpurun_out/r06_f_hostprof_medium.txt 2>&1 || exit 1
head -60 gpurun_out/r06_f_hostprof_medium.txt

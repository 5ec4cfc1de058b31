set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof3 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe > $R/gpurun_out/prof3.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --eager --no-cpu-baseline --no-probe > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --eager --no-cpu-baseline --no-probe > $R/gpurun_out/pmc_write.log 2>&1

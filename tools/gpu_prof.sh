# rocprofv3: kernel stats of the bench (graph replay, 1 warmup + 3 timed) + FETCH_SIZE / WRITE_SIZE
# passes over one eager step (separate runs, as MI355X_MICROARCH.md prescribes)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof3 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-dead-block-line > $R/gpurun_out/prof3.log 2>&1
tail -1 $R/gpurun_out/prof3.log | cut -c1-200
if [ "$1" = "pmc" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --eager --no-cpu-baseline --no-probe --no-dead-block-line --no-optimizer > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --eager --no-cpu-baseline --no-probe --no-dead-block-line --no-optimizer > $R/gpurun_out/pmc_write.log 2>&1
fi
echo prof done

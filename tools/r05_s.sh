set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r05_s_suite.log 2>&1 || { rc=$?; tail -30 gpurun_out/r05_s_suite.log; [ $rc -le 1 ] || exit 1; }
tail -2 gpurun_out/r05_s_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 600 python -u bench.py > gpurun_out/r05_s_bench.json 2> gpurun_out/r05_s_bench.err || { tail -20 gpurun_out/r05_s_bench.err; exit 1; }
cut -c1-300 gpurun_out/r05_s_bench.json
bash tools/gpu_prof.sh r05_s
python3 tools/replay_step.py gpurun_out/prof_r05_s/run_kernel_trace.csv r05_s > gpurun_out/r05_s_step.txt
head -12 gpurun_out/r05_s_step.txt

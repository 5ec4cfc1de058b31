set -e
# bench line + rocprofv3 kernel trace / stats of the headline step at HEAD (no test suite)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r05_aa_bench.json 2> gpurun_out/r05_aa_bench.err || { tail -20 gpurun_out/r05_aa_bench.err; exit 1; }
cut -c1-300 gpurun_out/r05_aa_bench.json
bash tools/gpu_prof.sh r05_aa
python3 tools/replay_step.py gpurun_out/prof_r05_aa/run_kernel_trace.csv r05_aa > gpurun_out/r05_aa_step.txt
head -45 gpurun_out/r05_aa_step.txt

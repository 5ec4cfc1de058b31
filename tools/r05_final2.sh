set -e
# End-of-round evidence, part 2: rocprofv3 kernel trace / stats of the headline step with the PMC passes (HBM
# traffic, MFMA busy), the replayed-step summary, and the small / medium config lines (HEAD tree)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05_fin}
PMC=1 bash tools/gpu_prof.sh $T
python3 tools/replay_step.py gpurun_out/prof_$T/run_kernel_trace.csv $T > gpurun_out/${T}_step.txt
head -8 gpurun_out/${T}_step.txt
timeout -k 10 600 python -u bench.py --config small --batch 8 --no-cpu-baseline > gpurun_out/${T}_small.json 2> gpurun_out/${T}_small.err || { tail -20 gpurun_out/${T}_small.err; exit 1; }
cut -c1-200 gpurun_out/${T}_small.json
timeout -k 10 600 python -u bench.py --config medium --batch 8 --no-cpu-baseline > gpurun_out/${T}_medium.json 2> gpurun_out/${T}_medium.err || { tail -20 gpurun_out/${T}_medium.err; exit 1; }
cut -c1-200 gpurun_out/${T}_medium.json
# host-bound configs: the same steps replayed from one captured graph (no per-launch host cost)
timeout -k 10 600 python -u bench.py --config small --batch 8 --no-cpu-baseline --graph --no-refpitch-line > gpurun_out/${T}_small_graph.json 2> gpurun_out/${T}_small_graph.err || { tail -20 gpurun_out/${T}_small_graph.err; exit 1; }
cut -c1-200 gpurun_out/${T}_small_graph.json
timeout -k 10 600 python -u bench.py --config medium --batch 8 --no-cpu-baseline --graph --no-refpitch-line > gpurun_out/${T}_medium_graph.json 2> gpurun_out/${T}_medium_graph.err || { tail -20 gpurun_out/${T}_medium_graph.err; exit 1; }
cut -c1-200 gpurun_out/${T}_medium_graph.json

set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python tools/phase_time.py > gpurun_out/phase.json 2> gpurun_out/phase.err || { tail -20 gpurun_out/phase.err; exit 1; }
cat gpurun_out/phase.json

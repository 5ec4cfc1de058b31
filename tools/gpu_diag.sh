set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/grad_diag.py variants > gpurun_out/grad_diag.jsonl 2> gpurun_out/grad_diag.err || { tail -20 gpurun_out/grad_diag.err; exit 1; }
cat gpurun_out/grad_diag.jsonl

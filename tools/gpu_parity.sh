set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread -k "attention or abby" > gpurun_out/t_attn.log 2>&1 || { tail -40 gpurun_out/t_attn.log; exit 1; }
tail -3 gpurun_out/t_attn.log
timeout -k 10 600 python -u tools/parity_probe.py > gpurun_out/parity_probe.jsonl 2> gpurun_out/parity_probe.err
cat gpurun_out/parity_probe.jsonl

set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r05_f_suite.log 2>&1 || { rc=$?; tail -40 gpurun_out/r05_f_suite.log; [ $rc -le 1 ] || exit 1; }
tail -3 gpurun_out/r05_f_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 600 python -u bench.py > gpurun_out/r05_f_bench.json 2> gpurun_out/r05_f_bench.err || { tail -20 gpurun_out/r05_f_bench.err; exit 1; }
cut -c1-400 gpurun_out/r05_f_bench.json
B="--no-cpu-baseline --no-dead-block-line --no-refpitch-line"
timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --precision fp32 $B > gpurun_out/r05_f_fp32.json 2> gpurun_out/r05_f_fp32.err
timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --precision x3 $B > gpurun_out/r05_f_x3.json 2> gpurun_out/r05_f_x3.err
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 $B --eager > gpurun_out/r05_f_eager.json 2> gpurun_out/r05_f_eager.err
bash tools/gpu_prof.sh r05_f
echo done

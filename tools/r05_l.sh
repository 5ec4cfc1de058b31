set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rot_fused.py -q -rf --timeout 120 --timeout-method thread > gpurun_out/r05_l_rot.log 2>&1 || { tail -30 gpurun_out/r05_l_rot.log; exit 1; }
tail -2 gpurun_out/r05_l_rot.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r05_l_suite.log 2>&1 || { rc=$?; tail -30 gpurun_out/r05_l_suite.log; [ $rc -le 1 ] || exit 1; }
tail -2 gpurun_out/r05_l_suite.log
B="--no-cpu-baseline --no-dead-block-line --no-refpitch-line --no-optimizer"
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 $B > gpurun_out/r05_l_bench.json 2>gpurun_out/r05_l_bench.err
cut -c1-300 gpurun_out/r05_l_bench.json
for t in med2 med8; do
  if [ $t = med2 ]; then b=2; else b=8; fi
  bash tools/gpu_prof.sh r05_l_$t --config medium --batch $b
  python3 tools/replay_step.py gpurun_out/prof_r05_l_$t/run_kernel_trace.csv $t > gpurun_out/r05_l_${t}_step.txt
  rm -f gpurun_out/prof_r05_l_$t/run_kernel_trace.csv
done
head -30 gpurun_out/r05_l_med8_step.txt

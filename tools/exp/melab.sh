set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_mel.py -k "logmel or mel" tests/test_golden.py > gpurun_out/mel_t.log 2>&1 || { tail -30 gpurun_out/mel_t.log; exit 1; }
tail -2 gpurun_out/mel_t.log
for v in melold prod; do
  if [ $v = prod ]; then L=""; else L=$PWD/tools/exp/libasrx_$v.so; fi
  echo "== $v"; ASRX_LIB=$L timeout -k 10 120 python tools/microbench.py mel 2>&1 | grep logmel
done

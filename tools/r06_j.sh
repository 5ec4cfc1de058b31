#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export GEMM_SHAPES="8192,384,384;8192,1152,384;8192,384,1152;2048,768,768;2048,2304,768;2048,768,2304;2048,1024,1024;2048,3072,1024"
for v in 5 0 2; do
  echo "variant $v"
  GEMM_VARIANT=$v GEMM_ITERS=100 timeout -k 10 200 python -u tools/gemm_micro.py 2>&1 | grep -v amdgpu.ids || exit 1
done

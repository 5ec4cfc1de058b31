set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_prof.sh r05_k_med2 --config medium --batch 2
bash tools/gpu_prof.sh r05_k_med8 --config medium --batch 8

set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_prof.sh r05_h_eager --eager

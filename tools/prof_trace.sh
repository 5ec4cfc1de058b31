# usage: bash tools/prof_trace.sh NAME [bench args...]  -> gpurun_out/NAME/ (kernel trace + stats)
set -e
NAME=$1; shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$NAME -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe "$@" > $R/gpurun_out/$NAME.log 2>&1

set -e
# End-of-round evidence, part 1: the whole -m gpu suite, smoke(), the default bench line (HEAD tree)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05_fin}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_suite.log 2>&1 || { rc=$?; tail -30 gpurun_out/${T}_suite.log; [ $rc -le 1 ] || exit 1; }
tail -2 gpurun_out/${T}_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
cut -c1-300 gpurun_out/${T}_bench.json

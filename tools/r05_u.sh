set -e
cd $GRAFT_REPO_ROOT
bash tools/r05_t.sh
bash tools/r05_s.sh

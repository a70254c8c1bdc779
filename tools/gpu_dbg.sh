set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/debug/airl_graph_dbg.py 2>&1 | grep -v Warn | tail -20

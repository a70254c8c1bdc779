set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cp}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python $GRAFT_REPO_ROOT/tools/conv_bench.py > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed rc=$?"; tail $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_$TAG -name "*.db" | head -1) 30 > gpurun_out/prof_${TAG}_summary.md
head -30 gpurun_out/prof_${TAG}_summary.md

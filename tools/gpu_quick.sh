# usage: bash tools/gpu_quick.sh TAG "pytest selection" [prof]
# selected GPU tests -> bench (20 steps) -> optional rocprofv3 kernel trace; stops at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-q}
SEL=${2:-tests}
if [ "$SEL" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $SEL -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_$TAG.log | head -30; tail -5 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_$TAG.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
if [ "$3" = "prof" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --eval-episodes 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed rc=$?"; exit 1; }
  cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_$TAG -name "*.db" | head -1) 40 > gpurun_out/prof_${TAG}_summary.md
  head -30 gpurun_out/prof_${TAG}_summary.md
fi
echo ALL OK

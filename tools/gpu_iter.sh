# Iteration loop on the GPU box: a pytest selection (default: the device-engine tests),
# then bench.py, then a rocprofv3 kernel-trace summary of the bench. Stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-it}
SEL=${2:-tests/engine}
timeout -k 10 400 python -u -m pytest $SEL -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed rc=$?"; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_$TAG -name "*.db" | head -1) 25 > gpurun_out/prof_${TAG}_summary.md
head -20 gpurun_out/prof_${TAG}_summary.md
echo ALL OK

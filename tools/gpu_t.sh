# targeted GPU tests ($1 = pytest selection) + 1-GPU bench; logs under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $1 -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_t.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_t.log | tail -20; exit 1; }
tail -2 gpurun_out/pytest_t.log
timeout -k 10 300 python bench.py > gpurun_out/bench_t.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_t.log; exit 1; }
tail -1 gpurun_out/bench_t.log

# quick GPU check: one-shot tests (block-count change), fused Adam, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/parallel/test_oneshot.py tests/ops/test_fused_adam.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_quick.log | tail -20; exit 1; }
tail -3 gpurun_out/pytest_quick.log
timeout -k 10 300 python bench.py > gpurun_out/bench_quick.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_quick.log; exit 1; }
tail -1 gpurun_out/bench_quick.log
echo ALL OK

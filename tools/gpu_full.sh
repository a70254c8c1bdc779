# full GPU test suite + smoke + 1-GPU bench (round-end rehearsal)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_gpu_full.log | tail -20; exit 1; }
tail -2 gpurun_out/pytest_gpu_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_full.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_full.log; exit 1; }
tail -1 gpurun_out/smoke_full.log
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
echo ALL OK

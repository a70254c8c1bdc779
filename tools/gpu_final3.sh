# session-3 end: new G > 16 PPO test cases, full GPU suite, smoke, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/engine/test_device_engine.py -m gpu -k "ppo_kernel_matches and g32 or ppo_kernel_matches and g64" > gpurun_out/f3_new.log 2>&1 || { echo "new tests failed"; tail -30 gpurun_out/f3_new.log; exit 1; }
tail -1 gpurun_out/f3_new.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/f3_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/f3_gpu.log; exit 1; }
tail -1 gpurun_out/f3_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f3_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/f3_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/f3_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/f3_bench.log; exit 1; }
tail -1 gpurun_out/f3_bench.log

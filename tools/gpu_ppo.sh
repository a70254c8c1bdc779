# PPO kernel numerics (single + cooperating workgroups), replicated-DP rehearsal on one card, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-ppo}
[ -n "$SKIP_PPO" ] || timeout -k 10 400 python -u -m pytest tests/engine/test_device_engine.py -x -v -m gpu -k ppo_kernel --timeout 120 --timeout-method thread > gpurun_out/pytest_ppo_$TAG.log 2>&1 || { echo "ppo tests failed rc=$?"; tail -40 gpurun_out/pytest_ppo_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_ppo_$TAG.log
timeout -k 10 400 python -u -m pytest tests/parallel/test_dist.py -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_dp_$TAG.log 2>&1 || { echo "dp tests failed rc=$?"; tail -40 gpurun_out/pytest_dp_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_dp_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
echo ALL OK

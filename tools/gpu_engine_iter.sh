# engine numerics (all device-engine GPU tests) + PPO probes + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-eng}
timeout -k 10 600 python -u -m pytest tests/engine -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_engine_$TAG.log 2>&1 || { echo "engine tests failed rc=$?"; tail -40 gpurun_out/pytest_engine_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_engine_$TAG.log
timeout -k 10 300 python -u tools/ppo_phase_probe.py > gpurun_out/phase_$TAG.log 2>&1 || { echo "phase probe failed"; tail -20 gpurun_out/phase_$TAG.log; exit 1; }
grep -v Warn gpurun_out/phase_$TAG.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
echo ALL OK

# PPO kernel iteration: numerics tests (single / cooperating workgroups, DP), phase + scale probes, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-iter}
timeout -k 10 400 python -u -m pytest tests/engine/test_device_engine.py -x -q -m gpu -k "ppo or overlap" --timeout 120 --timeout-method thread > gpurun_out/pytest_ppo_$TAG.log 2>&1 || { echo "ppo tests failed rc=$?"; tail -40 gpurun_out/pytest_ppo_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_ppo_$TAG.log
timeout -k 10 300 python -u tools/ppo_phase_probe.py > gpurun_out/phase_$TAG.log 2>&1 || { echo "phase probe failed"; tail -20 gpurun_out/phase_$TAG.log; exit 1; }
grep -v Warn gpurun_out/phase_$TAG.log | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/scale_$TAG.log 2>&1 || { echo "scale probe failed"; tail -20 gpurun_out/scale_$TAG.log; exit 1; }
grep -v Warn gpurun_out/scale_$TAG.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
echo ALL OK

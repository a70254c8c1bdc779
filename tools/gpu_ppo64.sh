# PPO kernel: correctness vs torch + GAIL / AIRL / DRLHP replicated-DP scale probes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/engine/test_device_engine.py -x -v -m gpu -k "ppo_kernel" --timeout 200 --timeout-method thread > gpurun_out/pytest_ppo64.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|passed|failed|assert" gpurun_out/pytest_ppo64.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_ppo64.log
for c in ${CONFIGS:-airl drlhp gail}; do
CONFIG=$c WS=${WS:-1,2,4,8} timeout -k 10 400 python -u tools/ppo_scale_probe.py > gpurun_out/probe_$c.log 2>&1 || { echo "$c probe failed"; tail -20 gpurun_out/probe_$c.log; exit 1; }
grep -v Warn gpurun_out/probe_$c.log | grep -v amdgpu.ids | grep -v "^    "
done
echo ALL OK

# optimizer / BC / pref / engine GPU tests, BC probe + trace, DAgger config line, PPO phase probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ops tests/algorithms tests/util tests/engine tests/parallel/test_oneshot.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r3b.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAILED|Error|error|passed|failed" gpurun_out/pytest_r3b.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r3b.log
bash tools/gpu_bc_prof.sh | head -30
CFGS=dagger_pong STEPS=2 timeout -k 10 600 bash tools/gpu_configs.sh r3b
timeout -k 10 300 python tools/ppo_phase_probe.py > gpurun_out/phase_r3b.log 2>&1 || { echo "phase probe failed"; tail -5 gpurun_out/phase_r3b.log; exit 1; }
cat gpurun_out/phase_r3b.log

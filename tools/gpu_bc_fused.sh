# fused CNN BC step: GPU tests, step probe, DAgger-Pong / all-config bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/algorithms/test_bc.py tests/util/test_networks.py tests/engine/test_device_dagger.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_bc.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAILED|Error|error|passed|failed" gpurun_out/pytest_bc.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_bc.log
timeout -k 10 200 python tools/bc_step_probe.py > gpurun_out/bc_probe.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/bc_probe.log; exit 1; }
cat gpurun_out/bc_probe.log | tail -2
CFGS=${CFGS:-dagger_pong,airl_hopper,preference_walker2d} STEPS=2 timeout -k 10 900 bash tools/gpu_configs.sh bcf

# net-split PPO: engine tests, bench (split on / off), phase probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/engine tests/rl > gpurun_out/pytest_ns.log 2>&1 || { echo "FAILED rc=$?"; grep -E "FAILED|Error|passed|failed|assert" gpurun_out/pytest_ns.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest_ns.log
timeout -k 10 300 python bench.py > gpurun_out/bench_ns.log 2>&1 && tail -1 gpurun_out/bench_ns.log | cut -c1-200
IMITATION_AMD_PPO_NETSPLIT=0 timeout -k 10 300 python bench.py > gpurun_out/bench_nons.log 2>&1 && tail -1 gpurun_out/bench_nons.log | cut -c1-200
CONFIG=gail timeout -k 10 300 python tools/ppo_scale_probe.py > gpurun_out/probe_ns.log 2>&1; tail -15 gpurun_out/probe_ns.log

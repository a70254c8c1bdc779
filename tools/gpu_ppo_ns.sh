# net-split PPO: engine tests, bench, scale probes (gail / airl / drlhp)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/engine tests/rl > gpurun_out/pytest_ns.log 2>&1 || { echo "FAILED rc=$?"; grep -E "FAILED|Error|passed|failed|assert" gpurun_out/pytest_ns.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_ns.log
timeout -k 10 300 python bench.py > gpurun_out/bench_ns.log 2>&1 && tail -1 gpurun_out/bench_ns.log | grep -o '"ms_per_step": [0-9.]*'
for c in gail airl drlhp; do
  CONFIG=$c timeout -k 10 400 python tools/ppo_scale_probe.py > gpurun_out/probe_ns_$c.log 2>&1 || { echo "probe $c failed"; tail -5 gpurun_out/probe_ns_$c.log; exit 1; }
  grep "ppo update" gpurun_out/probe_ns_$c.log
done

# BC head (bank-conflict-free) + Adam; XCD co-located PPO A/B (scale probe + bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/algorithms/test_bc.py tests/ops/test_kernels.py tests/engine/test_device_engine.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r3c.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAILED|Error|error|passed|failed" gpurun_out/pytest_r3c.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r3c.log
bash tools/gpu_bc_prof.sh | head -12
for x in 0 1; do
  IMITATION_AMD_PPO_XCD=$x CONFIG=gail timeout -k 10 300 python tools/ppo_scale_probe.py > gpurun_out/probe_xcd$x.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/probe_xcd$x.log; exit 1; }
  echo "XCD=$x"; grep "ppo update\|W=" gpurun_out/probe_xcd$x.log | head -8
  IMITATION_AMD_PPO_XCD=$x timeout -k 10 300 python bench.py > gpurun_out/bench_xcd$x.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_xcd$x.log; exit 1; }
  tail -1 gpurun_out/bench_xcd$x.log | grep -o '"ms_per_step": [0-9.]*'
done

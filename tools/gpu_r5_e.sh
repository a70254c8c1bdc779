#!/bin/bash
# round 5, call E: engine / DP / quality GPU tests, exchange-mask A/B (scale probe), bench
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/engine/test_device_engine.py -k "${ENGINE_K:-nan_reward or rollout_stats}" > gpurun_out/r5_e_engine.log 2>&1 &&
timeout -k 10 300 $T tests/engine/test_imitation_quality.py > gpurun_out/r5_e_quality.log 2>&1 &&
timeout -k 10 500 $T tests/parallel/test_oneshot.py > gpurun_out/r5_e_oneshot.log 2>&1 &&
for X in 1 0; do
  IMITATION_AMD_PPO_XMASK=$X WS=1,8 CONFIG=gail timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/r5_e_probe_gail_x$X.log 2>&1 || exit 1
  IMITATION_AMD_PPO_XMASK=$X WS=1,8 CONFIG=airl timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/r5_e_probe_airl_x$X.log 2>&1 || exit 1
done &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r5_e_bench.log 2>&1

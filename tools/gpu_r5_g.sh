#!/bin/bash
# round 5, call G: AIRL staging during PPO (bitwise tests + A/B), kernel profile of the headline bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/engine/test_device_engine.py -k "airl" > gpurun_out/r5_g_tests.log 2>&1 &&
timeout -k 10 400 $T tests/parallel/test_oneshot.py -k "airl" > gpurun_out/r5_g_oneshot.log 2>&1 &&
rm -f gpurun_out/r5_g_airl_ab.jsonl &&
for rep in 1 2; do
  for E in 0 1; do
    IMITATION_AMD_AIRL_EARLY_STAGE=$E timeout -k 10 200 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 10 --warmup 2 > gpurun_out/r5_g_airl_e$E.log 2>&1 || exit 1
    echo "{\"early\": $E, \"rep\": $rep, \"line\": $(grep '^{' gpurun_out/r5_g_airl_e$E.log | tail -1)}" >> gpurun_out/r5_g_airl_ab.jsonl || exit 1
  done
done &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_g_prof -o bench -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/r5_g_prof.log 2>&1

#!/bin/bash
# round 5, call H: device-scope stream events on the round's critical path (tests + A/B + trace)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/engine/test_device_engine.py -k "pipelined or overlap or rounds or resume or nan or rollout_stats or evaluate" > gpurun_out/r5_h_tests.log 2>&1 &&
rm -f gpurun_out/r5_h_ab.txt &&
for rep in 1 2; do
  for E in 0 1; do
    IMITATION_AMD_DEVICE_EVENTS=$E timeout -k 10 200 python -u bench.py --steps 40 --warmup 3 > gpurun_out/r5_h_bench_e$E.log 2>&1 || exit 1
    echo "bench events=$E rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_h_bench_e$E.log)" >> gpurun_out/r5_h_ab.txt || exit 1
    IMITATION_AMD_DEVICE_EVENTS=$E timeout -k 10 200 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 10 --warmup 2 > gpurun_out/r5_h_airl_e$E.log 2>&1 || exit 1
    echo "airl events=$E rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_h_airl_e$E.log)" >> gpurun_out/r5_h_ab.txt || exit 1
  done
done &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_h_prof -o bench -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/r5_h_prof.log 2>&1

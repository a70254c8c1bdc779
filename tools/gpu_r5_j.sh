#!/bin/bash
# round 5, call J: DAgger-Pong round -- runner reuse, async frame landing, async rollout stats,
# conv wgrads on parallel streams (A/B)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/engine/test_device_dagger.py tests/algorithms/test_bc.py tests/engine/test_device_engine.py -k "dagger or bc or airl_pipelined" -m gpu > gpurun_out/r5_j_tests.log 2>&1 &&
timeout -k 10 400 $T tests/parallel/test_oneshot.py -k "dagger or airl" > gpurun_out/r5_j_dp.log 2>&1 &&
IMITATION_AMD_BC_ASYNC_STATS=0 IMITATION_AMD_DAGGER_ASYNC_FRAMES=0 timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_j_dagger_sync.log 2>&1 &&
timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_j_dagger.log 2>&1 &&
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 5 --warmup 1 > gpurun_out/r5_j_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_j_prof -o dagger -- python3 tools/dagger_breakdown.py --rounds 2 --warmup 1 > gpurun_out/r5_j_prof.log 2>&1

#!/bin/bash
# round 5, call N: BC epoch step with the step-counter add and metrics append folded into existing launches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/engine/test_device_dagger.py tests/algorithms/test_bc.py tests/ops -m gpu > gpurun_out/r5_n_tests.log 2>&1 &&
IMITATION_AMD_BC_FOLD_LAUNCHES=0 timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_n_dagger_f0.log 2>&1 &&
timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_n_dagger.log 2>&1 &&
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 5 --warmup 1 > gpurun_out/r5_n_bench.log 2>&1

#!/bin/bash
# round 5, call S: DRLHP iteration after the fragmenter + gatherer changes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/pref_breakdown.py --iters 3 > gpurun_out/r5_s_pref.log 2>&1 &&
timeout -k 10 600 python -u benchmarking/bench_configs.py --configs preference_walker2d --steps 3 --warmup 1 > gpurun_out/r5_s_pref_bench.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/algorithms/test_preference_comparisons.py tests/engine -m gpu -k "pref or reward_model" > gpurun_out/r5_s_tests.log 2>&1

#!/bin/bash
# round 5, call AF: cnn_fc with 8 k-steps of loads in flight -- tests, kernel table, DAgger bench x2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/ops tests/engine/test_device_dagger.py tests/algorithms/test_dagger.py -m gpu > gpurun_out/r5_af_tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r5_af_prof -o run -- python3 tools/dagger_breakdown.py --rounds 2 > gpurun_out/r5_af_prof.log 2>&1 &&
timeout -k 10 120 python3 tools/prof_summary.py $(ls /tmp/r5_af_prof/*.db | head -1) > gpurun_out/r5_af_kernels.md && rm -rf /tmp/r5_af_prof &&
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 --out gpurun_out/r5_af_bench.jsonl > gpurun_out/r5_af_bench.log 2>&1 &&
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 --out gpurun_out/r5_af_bench.jsonl > gpurun_out/r5_af_bench2.log 2>&1

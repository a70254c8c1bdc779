#!/bin/bash
# round 5, call K: graph-replay boundary cost; DAgger collector head kernels (all loads in flight, heads on separate waves)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 120 python -u tools/graph_replay_probe.py --nodes 304 --reps 50 > gpurun_out/r5_k_graph304.log 2>&1 &&
timeout -k 10 120 python -u tools/graph_replay_probe.py --nodes 19 --reps 200 > gpurun_out/r5_k_graph19.log 2>&1 &&
timeout -k 10 600 $T tests/engine/test_device_dagger.py -m gpu > gpurun_out/r5_k_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_k_dagger.log 2>&1 &&
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 5 --warmup 1 > gpurun_out/r5_k_bench.log 2>&1

#!/bin/bash
# round 5, call V: BC epoch graphs replayed as two alternating instances (A/B), DAgger tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/engine/test_device_dagger.py tests/algorithms/test_bc.py -m gpu > gpurun_out/r5_v_tests.log 2>&1 &&
IMITATION_AMD_BC_GRAPH_PAIR=0 timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_v_dagger_p0.log 2>&1 &&
timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_v_dagger_p1.log 2>&1 &&
IMITATION_AMD_BC_GRAPH_PAIR=0 timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_v_dagger_p0b.log 2>&1 &&
timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_v_dagger_p1b.log 2>&1 &&
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 5 --warmup 1 > gpurun_out/r5_v_bench.log 2>&1

#!/bin/bash
# round 5, call Y: BC epoch graph size ladder (IMITATION_AMD_BC_GRAPH_K) -- bitwise tests, then A/B on DAgger-Pong
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/engine/test_device_dagger.py -m gpu > gpurun_out/r5_y_tests.log 2>&1 &&
for k in 16 64 32 16 64; do
  IMITATION_AMD_BC_GRAPH_K=$k timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 > gpurun_out/r5_y_k$k.log 2>&1 || exit 1
  tail -1 gpurun_out/r5_y_k$k.log >> gpurun_out/r5_y_ab.jsonl
  echo "k=$k done"
done &&
IMITATION_AMD_BC_GRAPH_K=64 timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 5 --warmup 1 > gpurun_out/r5_y_bench64.log 2>&1 &&
IMITATION_AMD_BC_GRAPH_K=16 timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 5 --warmup 1 > gpurun_out/r5_y_bench16.log 2>&1

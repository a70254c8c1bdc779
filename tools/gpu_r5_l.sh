#!/bin/bash
# round 5, call L: BC CNN step kernels (fc_wgrad 64-column blocks, prefetching conv dgrad, batched
# wgrad staging loads): numerics tests, DAgger A/B, kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/ops/test_conv.py tests/engine/test_device_dagger.py tests/algorithms/test_bc.py -m gpu > gpurun_out/r5_l_tests.log 2>&1 &&
IMITATION_AMD_CONV_DGRAD_PF=0 timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_l_dagger_pf0.log 2>&1 &&
timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_l_dagger.log 2>&1 &&
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 5 --warmup 1 > gpurun_out/r5_l_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_l_prof -o dagger -- python3 tools/dagger_breakdown.py --rounds 2 --warmup 1 > gpurun_out/r5_l_prof.log 2>&1

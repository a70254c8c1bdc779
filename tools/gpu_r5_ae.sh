#!/bin/bash
# round 5, call AE: conv forward with 8 k-steps of loads in flight; fc_wgrad bias lanes with their loads in flight -- tests, kernel table, DAgger bench;
# AIRL with / without the GC freeze (no regression check)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/ops/test_conv.py tests/algorithms/test_bc.py tests/engine/test_device_dagger.py -m gpu > gpurun_out/r5_ae_tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r5_ae_prof -o run -- python3 tools/dagger_breakdown.py --rounds 2 > gpurun_out/r5_ae_prof.log 2>&1 &&
timeout -k 10 120 python3 tools/prof_summary.py $(ls /tmp/r5_ae_prof/*.db | head -1) > gpurun_out/r5_ae_kernels.md && rm -rf /tmp/r5_ae_prof &&
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 --out gpurun_out/r5_ae_bench.jsonl > gpurun_out/r5_ae_bench.log 2>&1 &&
for m in 1 0 1 0; do
  IMITATION_AMD_GC_FREEZE=$m timeout -k 10 300 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 10 --warmup 2 > gpurun_out/r5_ae_airl_g$m.log 2>&1 || exit 1
  grep '"value"' gpurun_out/r5_ae_airl_g$m.log | sed "s/^{/{\"gc_freeze\": $m, /" >> gpurun_out/r5_ae_airl.jsonl
done

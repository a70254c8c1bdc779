#!/bin/bash
# round 5, call AU: top-conv ReLU mask applied once in fc_dgrad's store -- bitwise tests, kernel table, DAgger A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/algorithms/test_bc.py tests/ops/test_conv.py tests/engine/test_device_dagger.py tests/ops/test_fused_adam.py -m gpu > gpurun_out/r5_au_tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r5_au_prof -o run -- python3 tools/dagger_breakdown.py --rounds 2 > gpurun_out/r5_au_prof.log 2>&1 &&
timeout -k 10 120 python3 tools/prof_summary.py $(ls /tmp/r5_au_prof/*.db | head -1) > gpurun_out/r5_au_kernels.md && rm -rf /tmp/r5_au_prof &&
for v in 1 0 1 0; do
  IMITATION_AMD_BC_MASK_DX=$v timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 > gpurun_out/r5_au_m$v.log 2>&1 || exit 1
  grep '"value"' gpurun_out/r5_au_m$v.log | sed "s/^{/{\"mask_dx\": $v, /" >> gpurun_out/r5_au_ab.jsonl
  echo "mask=$v done"
done

#!/bin/bash
# round 5, call AK: DAgger BC rollout statistics in line vs on the twin beside the epoch (A/B, 3 reps)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0 1 0 1 0; do
  IMITATION_AMD_BC_ASYNC_STATS=$v timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 > gpurun_out/r5_ak_a$v.log 2>&1 || exit 1
  grep '"value"' gpurun_out/r5_ak_a$v.log | sed "s/^{/{\"async_stats\": $v, /" >> gpurun_out/r5_ak_ab.jsonl
  echo "async=$v done"
done

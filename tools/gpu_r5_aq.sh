#!/bin/bash
# round 5, call AQ: AIRL alone in a process vs after GAIL in the same process (bench_configs), 2 reps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 3 --warmup 1 --out gpurun_out/r5_aq_alone.jsonl > gpurun_out/r5_aq_alone$r.log 2>&1 || exit 1
  timeout -k 10 300 python -u benchmarking/bench_configs.py --configs gail_halfcheetah,airl_hopper --steps 3 --warmup 1 --out gpurun_out/r5_aq_after.jsonl > gpurun_out/r5_aq_after$r.log 2>&1 || exit 1
  timeout -k 10 300 python -u benchmarking/bench_configs.py --configs bc_cartpole,airl_hopper --steps 3 --warmup 1 --out gpurun_out/r5_aq_afterbc.jsonl > gpurun_out/r5_aq_afterbc$r.log 2>&1 || exit 1
done

#!/bin/bash
# round 5, call AI: DAgger collect host profile (cProfile of the timed rounds); AIRL bench_configs vs warm-up length
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 3 --profile > gpurun_out/r5_ai_dagger_prof.log 2>&1 &&
for w in 1 3; do
  timeout -k 10 300 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 3 --warmup $w > gpurun_out/r5_ai_airl_w$w.log 2>&1 || exit 1
done &&
timeout -k 10 300 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 10 --warmup 1 > gpurun_out/r5_ai_airl_s10.log 2>&1

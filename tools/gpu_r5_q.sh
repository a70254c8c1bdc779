#!/bin/bash
# round 5, call Q: DP rehearsals on one card (2 ranks, gloo bootstrap + one-shot all-reduce) of the
# headline bench and the AIRL config; DRLHP iteration breakdown
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
IMITATION_AMD_DIST_BACKEND=gloo IMITATION_AMD_ONESHOT=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/r5_q_bench_dp2.log 2>&1 &&
IMITATION_AMD_DIST_BACKEND=gloo IMITATION_AMD_ONESHOT=1 timeout -k 10 400 python -u benchmarking/bench_configs.py --configs airl_hopper --gpus 2 --steps 4 --warmup 1 > gpurun_out/r5_q_airl_dp2.log 2>&1 &&
timeout -k 10 600 python -u tools/pref_breakdown.py --iters 3 > gpurun_out/r5_q_pref.log 2>&1

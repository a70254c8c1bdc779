#!/bin/bash
# round 5, call O: AIRL Hopper round kernel trace (early staging), DRLHP iteration
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_o_prof -o airl -- python3 benchmarking/bench_configs.py --configs airl_hopper --steps 6 --warmup 2 > gpurun_out/r5_o_prof.log 2>&1 &&
timeout -k 10 600 python -u benchmarking/bench_configs.py --configs preference_walker2d --steps 3 --warmup 1 > gpurun_out/r5_o_pref.log 2>&1

#!/bin/bash
# round 5, call R: DRLHP iteration after the fragmenter change; DAgger collect() host sections
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/pref_breakdown.py --iters 3 > gpurun_out/r5_r_pref.log 2>&1 &&
timeout -k 10 600 python -u benchmarking/bench_configs.py --configs preference_walker2d --steps 3 --warmup 1 > gpurun_out/r5_r_pref_bench.log 2>&1 &&
timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_r_dagger.log 2>&1

#!/bin/bash
# round 5, call T: DAgger collector host/GPU interplay (HIP API + kernel trace, one timed round)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/r5_t_prof -o dagger -- python3 tools/dagger_breakdown.py --rounds 1 --warmup 1 > gpurun_out/r5_t_prof.log 2>&1

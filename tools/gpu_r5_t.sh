#!/bin/bash
# round 5, call T: DRLHP phase thread-time; DAgger collector host/GPU interplay (HIP API + kernel trace,
# analysed on the box: the database itself is too large to copy back)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/pref_breakdown.py --iters 3 > gpurun_out/r5_t_pref.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d /tmp/r5_t_prof -o dagger -- python3 tools/dagger_breakdown.py --rounds 1 --warmup 1 > gpurun_out/r5_t_prof.log 2>&1 &&
timeout -k 10 120 python -u tools/dagger_api_gaps.py $(ls /tmp/r5_t_prof/*.db | head -1) 300 > gpurun_out/r5_t_api_gaps.txt 2>&1
rc=$?
rm -rf /tmp/r5_t_prof
exit $rc

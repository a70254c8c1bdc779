#!/bin/bash
# round 5, call T2: DAgger collector host/GPU interplay in the timed rounds (analysed on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d /tmp/r5_t2_prof -o dagger -- python3 tools/dagger_breakdown.py --rounds 2 --warmup 1 > gpurun_out/r5_t2_prof.log 2>&1 &&
timeout -k 10 120 python -u tools/dagger_api_gaps.py $(ls /tmp/r5_t2_prof/*.db | head -1) 200 > gpurun_out/r5_t2_api_gaps.txt 2>&1
rc=$?
rm -rf /tmp/r5_t2_prof
exit $rc

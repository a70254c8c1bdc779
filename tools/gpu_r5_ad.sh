#!/bin/bash
# round 5, call AD: channel-aligned fc_wgrad blocks -- bitwise / fp64 tests, kernel time, DAgger-Pong A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/ops/test_conv.py -k fc -m gpu > gpurun_out/r5_ad_tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r5_ad_prof -o run -- python3 tools/dagger_breakdown.py --rounds 2 > gpurun_out/r5_ad_prof.log 2>&1 &&
timeout -k 10 120 python3 tools/prof_summary.py $(ls /tmp/r5_ad_prof/*.db | head -1) > gpurun_out/r5_ad_kernels.md && rm -rf /tmp/r5_ad_prof &&
for v in 1 0 1 0; do
  IMITATION_AMD_FC_WGRAD_CH=$v timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 > gpurun_out/r5_ad_ch$v.log 2>&1 || exit 1
  tail -1 gpurun_out/r5_ad_ch$v.log | sed "s/^{/{\"ch\": $v, /" >> gpurun_out/r5_ad_ab.jsonl
  echo "ch=$v done"
done

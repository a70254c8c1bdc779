#!/bin/bash
# round 5, call Z: DRLHP agent rounds log one round late (no host gap between update and next rollout);
# GC pause accounting in the DRLHP breakdown
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/engine/test_device_preference.py -m gpu > gpurun_out/r5_z_tests.log 2>&1 &&
for m in 1 0 1 0; do
  IMITATION_AMD_PREF_DEFER_LOG=$m timeout -k 10 400 python -u tools/pref_breakdown.py --iters 4 > gpurun_out/r5_z_pref_d$m.log 2>&1 || exit 1
  (echo -n "{\"defer\": $m, \"r\": "; tail -1 gpurun_out/r5_z_pref_d$m.log; echo "}") >> gpurun_out/r5_z_ab.jsonl
  echo "defer=$m done"
done

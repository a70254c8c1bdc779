#!/bin/bash
# round 6 call I: row-form (LDS-free) rollout actor -- bitwise tests, phase breakdown, bench; one-launch
# weight packing (BC step); DAgger DP test on the epoch runner; AIRL CLI chunking check, DRLHP resume trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
  tests/engine/test_rollout_probe.py tests/ops/test_conv.py tests/engine/test_device_engine.py \
  "tests/parallel/test_oneshot.py::test_dagger_dp_fused_bc_step_matches_eager_dp" \
  > gpurun_out/r6i_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/rollout_breakdown.py > gpurun_out/r6i_breakdown.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > gpurun_out/r6i_bench.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/bc_step_probe.py > gpurun_out/r6i_bcstep.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/cli_resume_diag.py airl --chunks > gpurun_out/r6i_diag_airl_chunks.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/cli_resume_diag.py pref > gpurun_out/r6i_diag_pref.log 2>&1 || exit $?

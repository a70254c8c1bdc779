#!/bin/bash
# round 6 call H: rollout-chain phase clock (bitwise test + breakdown), DP BC epoch graphs with the
# overlapped FC all-reduce (bitwise vs the per-minibatch DP step), fail-fast / DRLHP agent resume GPU tests,
# device CLI resume divergence (AIRL, DRLHP)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
  tests/engine/test_rollout_probe.py tests/algorithms/test_fail_fast.py tests/engine/test_device_preference.py \
  "tests/parallel/test_oneshot.py::test_bc_dp_epoch_graphs_are_bitwise_the_per_minibatch_dp_step" \
  "tests/parallel/test_oneshot.py::test_dagger_dp_fused_bc_step_matches_eager_dp" \
  > gpurun_out/r6h_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/rollout_breakdown.py > gpurun_out/r6h_breakdown.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/cli_resume_diag.py airl > gpurun_out/r6h_diag_airl.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/cli_resume_diag.py pref > gpurun_out/r6h_diag_pref.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ops/test_conv.py > gpurun_out/r6h_conv_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6h_bcprof -o bc -- python3 $GRAFT_REPO_ROOT/tools/bc_step_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r6h_bcprof.log 2>&1 || exit $?

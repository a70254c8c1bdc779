#!/bin/bash
# round 6 call G: paired conv backward (tests, BC step A/B, DAgger reference schedule), shared side
# streams vs the alternating-instance slowdown, device CLI determinism (zero-policy demos, DRLHP)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/ops/test_conv.py tests/engine/test_device_dagger.py tests/algorithms/test_bc.py tests/scripts/test_cli_resume.py \
  > gpurun_out/r6g_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for f in 0 1; do IMITATION_AMD_BC_CONV_PAIR=$f timeout -k 10 120 python -u tools/bc_step_probe.py >> gpurun_out/r6g_bcstep.log 2>&1 || exit $?; done
timeout -k 10 300 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 --out gpurun_out/r6g_dagger_ref.jsonl > gpurun_out/r6g_dagger.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/alt_slow_probe.py > gpurun_out/r6g_alt.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/cli_resume_diag.py pref > gpurun_out/r6g_resume_diag_pref.log 2>&1 || exit $?
timeout -k 10 120 python -u bench.py > gpurun_out/r6g_bench.log 2>&1 || exit $?

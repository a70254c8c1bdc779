#!/bin/bash
# round 6 call E: fused-Adam BC step tests + A/B, DAgger reference-schedule baseline, CLI resume
# diagnosis, the alternating-instance slowdown under a kernel trace, device AIRL Pendulum seeds
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/engine/test_device_dagger.py tests/algorithms/test_bc.py tests/ops/test_conv.py \
  "tests/engine/test_device_preference.py::test_device_agent_checkpoint_resume_is_bitwise" \
  "tests/scripts/test_cli_resume.py::test_train_preference_comparisons_resume_is_bitwise_on_device" \
  > gpurun_out/r6e_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for f in 0 1; do IMITATION_AMD_BC_FUSED_ADAM=$f timeout -k 10 120 python -u tools/bc_step_probe.py >> gpurun_out/r6e_bcstep.log 2>&1 || exit $?; done
for f in 0 1; do IMITATION_AMD_BC_FUSED_ADAM=$f timeout -k 10 300 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 --out gpurun_out/r6e_dagger_ref_fused$f.jsonl >> gpurun_out/r6e_dagger.log 2>&1 || exit $?; done
timeout -k 10 300 python -u tools/cli_resume_diag.py gail > gpurun_out/r6e_resume_diag.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/r6e_alt -o run -- python3 $R/tools/alt_slow_probe.py > $R/gpurun_out/r6e_alt.log 2>&1 || exit $?
cd $R && timeout -k 10 60 python3 tools/alt_slow_probe.py --split $(find /tmp/r6e_alt -name "*kernel_trace.csv" | head -1) > gpurun_out/r6e_alt_split.md 2>&1 || exit $?
OUT=gpurun_out/r6e_airl_device.jsonl timeout -k 10 300 python -u tools/quality_probe.py airl:pendulum:1000000:0:512 airl:pendulum:1000000:0:8192 airl:pendulum:1000000:1:512 airl:pendulum:1000000:1:8192 > gpurun_out/r6e_airl.log 2>&1 || exit $?

#!/bin/bash
# round 6 call F: split-tap conv dgrad (tests, BC step A/B, DAgger reference schedule), device CLI
# determinism / resume diagnosis, the alternating-instance slowdown with a HIP API trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/engine/test_device_dagger.py tests/algorithms/test_bc.py tests/ops/test_conv.py \
  "tests/engine/test_device_preference.py::test_device_agent_checkpoint_resume_is_bitwise" \
  > gpurun_out/r6f_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for f in 0 1; do IMITATION_AMD_CONV_DGRAD_SPLIT=$f timeout -k 10 120 python -u tools/bc_step_probe.py >> gpurun_out/r6f_bcstep.log 2>&1 || exit $?; done
timeout -k 10 300 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 --out gpurun_out/r6f_dagger_ref_split.jsonl > gpurun_out/r6f_dagger.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/cli_resume_diag.py gail --deterministic > gpurun_out/r6f_resume_diag_det.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --output-format csv -d /tmp/r6f_alt -o run -- python3 $R/tools/alt_slow_probe.py > $R/gpurun_out/r6f_alt.log 2>&1 || exit $?
cd $R && timeout -k 10 120 python3 tools/alt_slow_probe.py --split $(find /tmp/r6f_alt -name "*kernel_trace.csv" | head -1) $(find /tmp/r6f_alt -name "*hip_api_trace.csv" | head -1) > gpurun_out/r6f_alt_split.md 2>&1
ls /tmp/r6f_alt/* >> gpurun_out/r6f_alt_split.md 2>&1

#!/bin/bash
# round 6 call D: remaining new GPU tests (CLI / engine resume, fail-fast), then the in-process probe
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/scripts/test_cli_resume.py tests/algorithms/test_fail_fast.py \
  "tests/engine/test_device_dagger.py::test_device_dagger_full_checkpoint_resume_is_bitwise" \
  "tests/engine/test_device_preference.py::test_device_agent_checkpoint_resume_is_bitwise" \
  -m gpu > gpurun_out/r6d_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/expert_inproc_probe.py > gpurun_out/r6d_probe.log 2>&1 || exit $?
exit $rc

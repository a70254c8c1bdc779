#!/bin/bash
# round 6 call C: new GPU tests (bench quality phase, CLI / engine resume), then the in-process probe
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_bench_contract.py tests/scripts/test_cli_resume.py \
  "tests/engine/test_device_dagger.py::test_device_dagger_full_checkpoint_resume_is_bitwise" \
  "tests/engine/test_device_preference.py::test_device_agent_checkpoint_resume_is_bitwise" \
  -m gpu > gpurun_out/r6c_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/expert_inproc_probe.py > gpurun_out/r6c_probe.log 2>&1 || exit $?

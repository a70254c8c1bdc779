#!/bin/bash
# round 6 call M: observation from registers (no LDS) for the HalfCheetah row-form chain -- bitwise test
# vs the LDS forms, phase breakdown, engine tests, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/engine/test_rollout_probe.py tests/engine/test_device_engine.py tests/test_bench_contract.py \
  > gpurun_out/r6m_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/rollout_breakdown.py > gpurun_out/r6m_breakdown.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > gpurun_out/r6m_bench.log 2>&1 || exit $?

#!/bin/bash
# round 6 call Z: contraction-explicit Adam update (folded-reduction blocks bitwise the elementwise path):
# Adam / BC / DAgger / one-shot DP tests, BC step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ops/test_fused_adam.py \
  tests/algorithms tests/engine/test_device_dagger.py tests/parallel/test_oneshot.py > gpurun_out/r6z_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do timeout -k 10 120 python -u tools/bc_step_probe.py >> gpurun_out/r6z_bcstep.log 2>&1 || exit $?; done

#!/bin/bash
# round 6 call AP: the BC epoch's Adam without the gradient-zeroing stores -- Adam / BC / DAgger / DP tests,
# BC step x3, kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ops/test_fused_adam.py \
  tests/algorithms/test_bc.py tests/engine/test_device_dagger.py tests/parallel/test_oneshot.py > gpurun_out/r6ap_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do timeout -k 10 120 python -u tools/bc_step_probe.py >> gpurun_out/r6ap_bcstep.log 2>&1 || exit $?; done
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6ap_bcprof -o bc -- python3 $R/tools/bc_step_probe.py > $R/gpurun_out/r6ap_bcprof.log 2>&1

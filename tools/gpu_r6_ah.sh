#!/bin/bash
# round 6 call AH: conv2's backward forked onto two streams (wgrad partials || split-tap dgrad) instead of the
# occupancy-starved paired launch: conv / BC / DAgger / DP tests, BC step A/B (interleaved), kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ops/test_conv.py \
  tests/algorithms/test_bc.py tests/engine/test_device_dagger.py tests/parallel/test_oneshot.py > gpurun_out/r6ah_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  for f in "" "--no-fork"; do
    timeout -k 10 120 python -u tools/bc_step_probe.py $f >> gpurun_out/r6ah_bcstep.log 2>&1 || exit $?
  done
done
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6ah_bcprof -o bc -- python3 $R/tools/bc_step_probe.py > $R/gpurun_out/r6ah_bcprof.log 2>&1

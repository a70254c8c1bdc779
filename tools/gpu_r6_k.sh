#!/bin/bash
# round 6 call K: one-launch weight packing with coalesced t_hwc tiles (test + BC-step trace), the
# two-wave hand-off probe
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ops/test_conv.py \
  tests/algorithms/test_bc.py > gpurun_out/r6k_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6k_bcprof -o bc -- python3 $GRAFT_REPO_ROOT/tools/bc_step_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r6k_bcprof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/wave_handoff_probe tools/wave_handoff_probe.hip && timeout -k 10 60 /tmp/wave_handoff_probe > gpurun_out/r6k_handoff.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/bc_step_probe.py > gpurun_out/r6k_bcstep.log 2>&1 || exit $?

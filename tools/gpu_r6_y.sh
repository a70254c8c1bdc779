#!/bin/bash
# round 6 call Y: conv weight-gradient reductions folded into the BC step's Adam launch (12 launches):
# tests, BC step A/B against the separate launches (interleaved), weight-gradient block cap 2M vs 4M
# partial floats (ab/cap4m.so), kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ops/test_fused_adam.py \
  tests/ops/test_conv.py tests/algorithms/test_bc.py tests/engine/test_device_dagger.py tests/parallel/test_oneshot.py \
  > gpurun_out/r6y_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  for f in "" "--sep-reduce" "--sep-gather --sep-reduce"; do
    timeout -k 10 120 python -u tools/bc_step_probe.py $f >> gpurun_out/r6y_bcstep.log 2>&1 || exit $?
  done
done
SO=imitation_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/orig.so
for v in cap4m fold cap4m fold; do
  cp ab/$v.so $SO
  echo "== $v" >> gpurun_out/r6y_bcstep.log
  timeout -k 10 120 python -u tools/bc_step_probe.py >> gpurun_out/r6y_bcstep.log 2>&1 || { cp /tmp/orig.so $SO; exit 1; }
done
cp /tmp/orig.so $SO
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6y_bcprof -o bc -- python3 $R/tools/bc_step_probe.py > $R/gpurun_out/r6y_bcprof.log 2>&1

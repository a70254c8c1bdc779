#!/bin/bash
# round 6 call T: A/B of the FC weight-gradient split over HW positions (1 / 2 / 4 blocks per channel
# group and n block): bitwise test vs the column blocks, fused BC step test, BC step time
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SO=imitation_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/orig.so
for v in 1 2 4 1 2 4; do
  cp ab/fcsplit$v.so $SO
  echo "== split $v" >> gpurun_out/r6t.log
  timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ops/test_conv.py -k "fc_wgrad" \
    tests/algorithms/test_bc.py -k "fc_wgrad or fused_cnn_bc_step" >> gpurun_out/r6t.log 2>&1
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then cp /tmp/orig.so $SO; exit $rc; fi
  timeout -k 10 120 python -u tools/bc_step_probe.py >> gpurun_out/r6t.log 2>&1 || { cp /tmp/orig.so $SO; exit 1; }
done
cp /tmp/orig.so $SO

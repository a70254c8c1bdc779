#!/bin/bash
# round 6 call U: A/B of the BC head's W columns in registers, and Adam's bias corrections once per block
# (baseline = fcsplit1, + head = head_new, + Adam = adam_v2): tests + BC step per variant, interleaved
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SO=imitation_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/orig.so
for v in fcsplit1 head_new adam_v2 fcsplit1 head_new adam_v2; do
  cp ab/$v.so $SO
  echo "== $v" >> gpurun_out/r6u.log
  timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/algorithms/test_bc.py \
    tests/ops/test_fused_adam.py >> gpurun_out/r6u.log 2>&1
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then cp /tmp/orig.so $SO; exit $rc; fi
  timeout -k 10 120 python -u tools/bc_step_probe.py >> gpurun_out/r6u.log 2>&1 || { cp /tmp/orig.so $SO; exit 1; }
done
cp /tmp/orig.so $SO

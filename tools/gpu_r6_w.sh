#!/bin/bash
# round 6 call W: row-form weight packing (rowpack); FC backward pair (as committed / data-gradient blocks first at <= 128 VGPRs / two launches)
# with the minibatch gather inside the weight-packing launch; fused vs separate gather. Tests per variant,
# BC step interleaved, then a kernel trace of the current build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
SO=imitation_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/orig.so
L=gpurun_out/r6w.log
for v in rowpack merge_pairfix merge_pair merge_nopair; do
  cp ab/$v.so $SO
  echo "== tests $v" >> $L
  timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/algorithms/test_bc.py \
    tests/ops/test_conv.py tests/ops/test_fused_adam.py "tests/engine/test_device_dagger.py::test_bc_epoch_graph_matches_per_minibatch_path" >> $L 2>&1
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then cp /tmp/orig.so $SO; exit $rc; fi
done
for v in rowpack merge_pairfix merge_pair merge_nopair rowpack merge_pairfix merge_pair merge_nopair; do
  cp ab/$v.so $SO
  echo "== $v" >> $L
  timeout -k 10 120 python -u tools/bc_step_probe.py >> $L 2>&1 || { cp /tmp/orig.so $SO; exit 1; }
  timeout -k 10 120 python -u tools/bc_step_probe.py --sep-gather >> $L 2>&1 || { cp /tmp/orig.so $SO; exit 1; }
done
cp /tmp/orig.so $SO
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6w_bcprof -o bc -- python3 $R/tools/bc_step_probe.py > $R/gpurun_out/r6w_bcprof.log 2>&1

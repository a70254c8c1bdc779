#!/bin/bash
# round 6 call AO: split-tap data gradient without runtime integer divisions (div_new) vs before (div_old)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ops/test_conv.py \
  tests/algorithms/test_bc.py tests/engine/test_device_dagger.py tests/parallel/test_oneshot.py > gpurun_out/r6ao_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SO=imitation_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/orig.so
for v in div_new div_old div_new div_old div_new div_old; do
  cp ab/$v.so $SO
  echo "== $v" >> gpurun_out/r6ao_bcstep.log
  timeout -k 10 120 python -u tools/bc_step_probe.py >> gpurun_out/r6ao_bcstep.log 2>&1 || { cp /tmp/orig.so $SO; exit 1; }
done
cp /tmp/orig.so $SO
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6ao_bcprof -o bc -- python3 $R/tools/bc_step_probe.py > $R/gpurun_out/r6ao_bcprof.log 2>&1
cd $R && timeout -k 10 120 python -u tools/dgrad_form_probe.py > gpurun_out/r6ao_dgrad_forms.log 2>&1

#!/bin/bash
# round 6 call X: the kept BC build (two-launch FC backward, row-form packing with the minibatch gather in
# its launch): BC / conv / Adam / DAgger / DP tests, BC step x3, kernel trace, DAgger-Pong reference schedule
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ops tests/algorithms \
  tests/engine/test_device_dagger.py tests/parallel/test_oneshot.py > gpurun_out/r6x_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do timeout -k 10 120 python -u tools/bc_step_probe.py >> gpurun_out/r6x_bcstep.log 2>&1 || exit $?; done
timeout -k 10 300 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 --out gpurun_out/r6x_dagger.jsonl > gpurun_out/r6x_dagger.log 2>&1 || exit $?
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6x_bcprof -o bc -- python3 $R/tools/bc_step_probe.py > $R/gpurun_out/r6x_bcprof.log 2>&1 || exit $?
cd $R && timeout -k 10 120 python -u tools/dgrad_form_probe.py > $R/gpurun_out/r6x_dgrad_forms.log 2>&1

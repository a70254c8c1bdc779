#!/bin/bash
# round 6 call V: the combined BC build -- GPU tests of the BC / DAgger / conv / Adam / DP paths, BC step,
# DAgger-Pong reference schedule, BC kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ops tests/algorithms \
  tests/engine/test_device_dagger.py tests/parallel/test_oneshot.py > gpurun_out/r6v_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/bc_step_probe.py > gpurun_out/r6v_bcstep.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 --out gpurun_out/r6v_dagger.jsonl > gpurun_out/r6v_dagger.log 2>&1 || exit $?
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6v_bcprof -o bc -- python3 $R/tools/bc_step_probe.py > $R/gpurun_out/r6v_bcprof.log 2>&1 || exit $?

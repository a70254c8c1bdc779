#!/bin/bash
# round 6 call J: FusedAdam state_dict snapshot fix + host env mirrored at train end (device CLI resume
# tests), BC-step tests and kernel trace with the one-launch weight packing, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
  tests/scripts/test_cli_resume.py tests/ops/test_fused_adam.py tests/engine/test_device_preference.py \
  tests/algorithms/test_bc.py tests/engine/test_device_dagger.py tests/algorithms/test_fail_fast.py \
  > gpurun_out/r6j_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6j_bcprof -o bc -- python3 $GRAFT_REPO_ROOT/tools/bc_step_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r6j_bcprof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && timeout -k 10 200 python -u bench.py > gpurun_out/r6j_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 --out gpurun_out/r6j_dagger_ref.jsonl > gpurun_out/r6j_dagger.log 2>&1 || exit $?

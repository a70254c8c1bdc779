#!/bin/bash
# round 6 call Q: the conv tests / BC / DAgger GPU tests on the 2M wgrad cap, then every BASELINE config once
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ops/test_conv.py \
  tests/algorithms/test_bc.py tests/engine/test_device_dagger.py tests/parallel/test_oneshot.py > gpurun_out/r6q_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 1000 python -u benchmarking/bench_configs.py --configs all --out gpurun_out/r6q_configs.jsonl \
  > gpurun_out/r6q_configs.log 2>&1 || exit $?

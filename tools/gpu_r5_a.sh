#!/bin/bash
# round 5, call A: new engine GPU tests, imitation-quality probe, headline bench
set -o pipefail
mkdir -p gpurun_out
export OUT=gpurun_out/r5_quality.jsonl
rm -f $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/engine/test_device_engine.py \
  -k "evaluate or gae_scan or gail_rounds or disc_overlap or airl_rounds_train or airl_pipelined" > gpurun_out/r5_tests_a.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r5_bench_a.log 2>&1 &&
timeout -k 10 600 python -u tools/quality_probe.py ${SPECS:-gail:cartpole:200000 airl:cartpole:200000 gail:pendulum:400000 airl:pendulum:400000} > gpurun_out/r5_quality.log 2>&1

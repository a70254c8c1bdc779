#!/bin/bash
# round 6 call R: PPO prep kernel with batched row loads -- PPO / engine tests, kernel trace of the bench,
# bench, DRLHP PPO update
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/engine/test_device_engine.py \
  tests/parallel/test_oneshot.py > gpurun_out/r6r_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r6_r_kt -o run -- python3 $R/bench.py --steps 20 --warmup 3 --eval-episodes 0 > $R/gpurun_out/r6r_kt.log 2>&1 || exit $?
cd $R && cp $(find /tmp/r6_r_kt -name "*kernel_stats.csv" | head -1) gpurun_out/r6r_kernel_stats.csv && rm -rf /tmp/r6_r_kt
timeout -k 10 200 python -u bench.py > gpurun_out/r6r_bench.log 2>&1 || exit $?
CONFIG=drlhp WS=1 timeout -k 10 150 python -u tools/ppo_scale_probe.py > gpurun_out/r6r_drlhp.log 2>&1 || exit $?

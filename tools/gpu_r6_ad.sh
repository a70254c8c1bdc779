#!/bin/bash
# round 6 call AD: DAgger-Pong at the reference schedule (4 timed rounds), twice, with the round-end BC step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 \
    --out gpurun_out/r6ad_dagger.jsonl >> gpurun_out/r6ad_dagger.log 2>&1 || exit $?
done
timeout -k 10 120 python -u tools/bc_step_probe.py > gpurun_out/r6ad_bcstep.log 2>&1

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export OUT=gpurun_out/r5_quality2.jsonl
rm -f $OUT
timeout -k 10 900 python -u tools/quality_probe.py gail:cartpole:1000000:0 gail:cartpole:1000000:1 gail:cartpole:1000000:2 \
  airl:cartpole:2500000:0 airl:cartpole:2500000:0:16384 airl:cartpole:2500000:1:16384 \
  gail:pendulum:600000:0 gail:pendulum:600000:1 airl:pendulum:1000000:0 airl:pendulum:1000000:0:8192 > gpurun_out/r5_quality2.log 2>&1

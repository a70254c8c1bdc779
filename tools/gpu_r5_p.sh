#!/bin/bash
# round 5, call P: AIRL Pendulum discriminator schedule / reward normalisation sweep (1M steps each)
set -o pipefail
mkdir -p gpurun_out
export OUT=gpurun_out/r5_p_airl_pendulum.jsonl
rm -f $OUT
timeout -k 10 900 python -u tools/quality_probe.py \
  airl:pendulum:1000000:0:8192:16:2048:1 airl:pendulum:1000000:0:8192:4:2048:0 airl:pendulum:1000000:0:8192:4:2048:1 \
  airl:pendulum:1000000:0:8192:8:1024:1 airl:pendulum:1000000:0:512:4:1024:1 airl:pendulum:1000000:1:8192:4:2048:1 \
  > gpurun_out/r5_p_probe.log 2>&1

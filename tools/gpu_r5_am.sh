#!/bin/bash
# round 5, call AM: CLI train_adversarial speed with the training-loop GC freeze on / off
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in 1 0 1 0; do
  IMITATION_AMD_GC_FREEZE=$m timeout -k 10 400 python -u tools/cli_speed.py --rounds 60 --ckpt 10 > gpurun_out/r5_am_cli_g$m.log 2>&1 || exit 1
  tail -1 gpurun_out/r5_am_cli_g$m.log | sed "s/^{/{\"gc_freeze\": $m, /" >> gpurun_out/r5_am_ab.jsonl
  echo "freeze=$m done"
done

#!/bin/bash
# round 6 call L: PPO occupancy experiment -- the W = 1 update of the GAIL bench
# config and the DRLHP config over 1 / 2 / 4 cooperating workgroups per minibatch (row chunks of
# 64 / 32 / 16) and with / without the actor-critic net split; one process per setting
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6l_occupancy.log
: > $out
for cfg in gail drlhp; do
  for cw in 0 32 16; do
    echo "== CONFIG=$cfg RC_CW=$cw" >> $out
    CONFIG=$cfg WS=1 RC_CW=$cw timeout -k 10 150 python -u tools/ppo_scale_probe.py >> $out 2>&1 || exit $?
  done
  echo "== CONFIG=$cfg NETSPLIT=0" >> $out
  CONFIG=$cfg WS=1 IMITATION_AMD_PPO_NETSPLIT=0 timeout -k 10 150 python -u tools/ppo_scale_probe.py >> $out 2>&1 || exit $?
done

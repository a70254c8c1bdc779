#!/bin/bash
# round 5, call U: DRLHP / AIRL PPO plan alternatives (chunk width, cooperating-group cap)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in drlhp airl; do
  for v in "0 0" "32 0" "0 1" "0 4"; do
    set -- $v
    RC_CW=$1 RC_GMAX=$2 CONFIG=$c WS=1 timeout -k 10 200 python -u tools/ppo_scale_probe.py > gpurun_out/r5_u_${c}_cw$1_g$2.log 2>&1
    rc=$?
    if [ $rc -ge 124 ]; then echo "probe $c $v: rc $rc (timeout / crash): stopping"; exit $rc; fi
    [ $rc -ne 0 ] && echo "probe $c $v failed (rc $rc, plan rejected?)"
  done
done
exit 0

# XCD placement A/B for the 64-wide plans (airl / drlhp) and gail, scale probe W=1..8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in airl drlhp gail; do
  for x in 0 1; do
    IMITATION_AMD_PPO_XCD=$x IMITATION_AMD_PPO_XCHG2_SWEEP=0 CONFIG=$c timeout -k 10 400 python tools/ppo_scale_probe.py > gpurun_out/probe2_${c}_xcd$x.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/probe2_${c}_xcd$x.log; exit 1; }
    echo "$c XCD=$x"; grep "ppo update" gpurun_out/probe2_${c}_xcd$x.log
  done
done

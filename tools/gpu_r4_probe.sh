# round-4: per-phase PPO cycle counters (ppo_scale_probe) for the three headline plans
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CONFIG=gail WS=1,8 timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/r4p_gail.log 2>&1 || { echo "gail probe failed"; tail -20 gpurun_out/r4p_gail.log; exit 1; }
cat gpurun_out/r4p_gail.log | grep -v Warn
CONFIG=airl WS=1,8 timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/r4p_airl.log 2>&1 || { echo "airl probe failed"; tail -20 gpurun_out/r4p_airl.log; exit 1; }
cat gpurun_out/r4p_airl.log | grep -v Warn
CONFIG=drlhp WS=1 timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/r4p_drlhp.log 2>&1 || { echo "drlhp probe failed"; tail -20 gpurun_out/r4p_drlhp.log; exit 1; }
cat gpurun_out/r4p_drlhp.log | grep -v Warn

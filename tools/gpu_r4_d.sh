# round-4: DAgger-Pong phase probe; GAIL W=8 plan alternatives (net split off, G caps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dagger_probe.py > gpurun_out/r4d_dagger.log 2>&1 || { echo "dagger probe failed"; tail -30 gpurun_out/r4d_dagger.log; exit 1; }
grep -v Warn gpurun_out/r4d_dagger.log | head -60
for gm in 2 4; do
  CONFIG=gail WS=8 RC_GMAX=$gm timeout -k 10 200 python -u tools/ppo_scale_probe.py > gpurun_out/r4d_gail_g$gm.log 2>&1 || { echo "gmax probe failed"; tail -20 gpurun_out/r4d_gail_g$gm.log; exit 1; }
  grep "ppo update" gpurun_out/r4d_gail_g$gm.log
done
IMITATION_AMD_PPO_NETSPLIT=0 CONFIG=gail WS=1,8 timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/r4d_gail_nons.log 2>&1 || { echo "nons probe failed"; tail -20 gpurun_out/r4d_gail_nons.log; exit 1; }
grep "ppo update\|cycles" gpurun_out/r4d_gail_nons.log

# round-4: PPO probe after BF3 -- W=1/8 for the three plans, G caps at W=8, exclusive-LDS knob
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in gail airl drlhp; do
  CONFIG=$cfg WS=1,2,4,8 timeout -k 10 400 python -u tools/ppo_scale_probe.py > gpurun_out/r4q_$cfg.log 2>&1 || { echo "$cfg probe failed"; tail -20 gpurun_out/r4q_$cfg.log; exit 1; }
  grep -v Warn gpurun_out/r4q_$cfg.log
done
for gm in 2 4; do
  CONFIG=gail WS=8 RC_GMAX=$gm timeout -k 10 200 python -u tools/ppo_scale_probe.py > gpurun_out/r4q_gail_g$gm.log 2>&1 || { echo "gmax probe failed"; tail -20 gpurun_out/r4q_gail_g$gm.log; exit 1; }
  grep "ppo update" gpurun_out/r4q_gail_g$gm.log
done
IMITATION_AMD_PPO_NETSPLIT=0 CONFIG=gail WS=1,2,4,8 timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/r4q_gail_nons.log 2>&1 || { echo "nons probe failed"; tail -20 gpurun_out/r4q_gail_nons.log; exit 1; }
grep "ppo update\|cycles" gpurun_out/r4q_gail_nons.log
IMITATION_AMD_PPO_NETSPLIT=0 timeout -k 10 300 python bench.py > gpurun_out/r4q_bench_nons.log 2>&1 || { echo "bench nons failed"; tail -20 gpurun_out/r4q_bench_nons.log; exit 1; }
tail -1 gpurun_out/r4q_bench_nons.log
IMITATION_AMD_PPO_LDS_EXCL=1 timeout -k 10 300 python bench.py > gpurun_out/r4q_bench_excl.log 2>&1 || { echo "bench excl failed"; tail -20 gpurun_out/r4q_bench_excl.log; exit 1; }
tail -1 gpurun_out/r4q_bench_excl.log
timeout -k 10 300 python bench.py > gpurun_out/r4q_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r4q_bench.log; exit 1; }
tail -1 gpurun_out/r4q_bench.log
timeout -k 10 200 python -u tools/wlin_roofline.py > gpurun_out/r4q_wlin.md 2> gpurun_out/r4q_wlin.err || { echo "wlin roofline failed"; tail -20 gpurun_out/r4q_wlin.err; exit 1; }
cat gpurun_out/r4q_wlin.md

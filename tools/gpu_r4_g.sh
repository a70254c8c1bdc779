# round-4: rollout step-chain breakdown (GAIL / AIRL recipes) + headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in gail_halfcheetah airl_hopper; do
  RECIPE=$r timeout -k 10 200 python -u tools/rollout_probe.py > gpurun_out/r4g_$r.log 2>&1 || { echo "rollout probe failed"; tail -20 gpurun_out/r4g_$r.log; exit 1; }
  echo "== $r"; grep "chain\|cycles" gpurun_out/r4g_$r.log
done
timeout -k 10 300 python bench.py > gpurun_out/r4g_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r4g_bench.log; exit 1; }
tail -1 gpurun_out/r4g_bench.log | cut -c1-250

# one- vs two-level PPO partial exchange: GAIL replicated-DP scale probe + AIRL-Hopper config (G = 16 at W = 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/scale_probe.log 2>&1 || { echo "probe failed rc=$?"; tail -20 gpurun_out/scale_probe.log; exit 1; }
grep -v -i warn gpurun_out/scale_probe.log | grep -v amdgpu.ids
for x in 0 1; do
  IMITATION_AMD_PPO_XCHG2=$x timeout -k 10 300 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 3 --warmup 1 --eval-episodes 2 --out gpurun_out/airl_x$x.jsonl > gpurun_out/airl_x$x.log 2>&1 || { echo "airl failed rc=$?"; tail -20 gpurun_out/airl_x$x.log; exit 1; }
  echo "xchg2=$x"; cut -c1-260 gpurun_out/airl_x$x.jsonl
done

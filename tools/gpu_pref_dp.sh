# DRLHP-Walker config with 2 ranks on ONE GPU (gloo bootstrap): eager DP reward trainer
# (IMITATION_AMD_ONESHOT=0) vs graphed minibatches on the one-shot all-reduce (=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp IMITATION_AMD_DIST_BACKEND=gloo
for os in 0 1; do
  IMITATION_AMD_ONESHOT=$os timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29575 benchmarking/bench_configs.py --configs preference_walker2d --steps 2 --warmup 1 --eval-episodes 2 --out gpurun_out/pref_dp2_os$os.jsonl > gpurun_out/pref_dp2_os$os.log 2>&1 || { echo "pref dp2 oneshot=$os failed rc=$?"; tail -30 gpurun_out/pref_dp2_os$os.log; exit 1; }
  echo "oneshot=$os"; cut -c1-400 gpurun_out/pref_dp2_os$os.jsonl
done
echo ALL OK

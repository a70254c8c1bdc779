# 2- and 4-rank rehearsal of bench.py on ONE GPU (gloo backend: RCCL needs distinct devices)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp IMITATION_AMD_DIST_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus $n --steps 3 --warmup 1 --eval-episodes 2 > gpurun_out/dp$n.log 2>&1 || { echo "dp$n failed rc=$?"; tail -30 gpurun_out/dp$n.log; exit 1; }
  grep '"metric"' gpurun_out/dp$n.log | cut -c1-260
done
echo ALL OK

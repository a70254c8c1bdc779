# one-shot all-reduce: kernel / DP tests on one card, then the 2- and 4-rank bench rehearsal
# with the disc buckets on the one-shot path (gloo bootstrap, IMITATION_AMD_ONESHOT=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/parallel -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/oneshot_tests.log 2>&1 || { echo "tests failed"; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/oneshot_tests.log | tail -20; exit 1; }
grep -E "\{|passed" gpurun_out/oneshot_tests.log
export IMITATION_AMD_DIST_BACKEND=gloo IMITATION_AMD_ONESHOT=1
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus $n --steps 3 --warmup 1 --eval-episodes 2 > gpurun_out/dp${n}_oneshot.log 2>&1 || { echo "dp$n failed rc=$?"; tail -30 gpurun_out/dp${n}_oneshot.log; exit 1; }
  grep '"metric"' gpurun_out/dp${n}_oneshot.log | cut -c1-300
done
echo ALL OK

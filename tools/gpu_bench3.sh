# bench.py three times (variance check)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench3_$i.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench3_$i.log; exit 1; }
  tail -1 gpurun_out/bench3_$i.log | grep -o '"ms_per_step": [0-9.]*'
done

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pc}
CFGS=${CFGS:-airl_hopper}
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python $GRAFT_REPO_ROOT/benchmarking/bench_configs.py --configs $CFGS --steps 2 --warmup 1 --eval-episodes 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed rc=$?"; tail $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_$TAG -name "*.db" | head -1) 30 > gpurun_out/prof_${TAG}_summary.md
head -34 gpurun_out/prof_${TAG}_summary.md

# round-4: kernel trace of the AIRL Hopper config (one-round timeline -> prof_summary.py round)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/airltr -o p -- python3 benchmarking/bench_configs.py --configs airl_hopper --steps 3 --warmup 1 --eval-episodes 1 > gpurun_out/airltr.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/airltr.log; exit 1; }
echo trace ok

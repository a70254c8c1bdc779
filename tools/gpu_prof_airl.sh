# kernel trace of the AIRL-Hopper bench config
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_airl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_airl -o airl -- python3 benchmarking/bench_configs.py --configs airl_hopper --steps 3 --warmup 1 > gpurun_out/prof_airl.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_airl.log; exit 1; }
find gpurun_out/prof_airl -name "*kernel_stats.csv" | head -3
echo ALL OK

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/scripts/test_scripts.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/cli_gpu.log 2>&1 || { grep -E "Error|error|FAIL|assert" gpurun_out/cli_gpu.log | head -30; exit 1; }
tail -1 gpurun_out/cli_gpu.log
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 4 --warmup 1 --eval-episodes 0 > gpurun_out/airl_bench.log 2>&1 || { tail -20 gpurun_out/airl_bench.log; exit 1; }
grep config gpurun_out/airl_bench.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_airl -o run -- python $GRAFT_REPO_ROOT/benchmarking/bench_configs.py --configs airl_hopper --steps 3 --warmup 1 --eval-episodes 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_airl.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_airl.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_airl -name "*.db" | head -1) 40 > gpurun_out/prof_airl_summary.md
rm -rf gpurun_out/prof_airl
head -30 gpurun_out/prof_airl_summary.md

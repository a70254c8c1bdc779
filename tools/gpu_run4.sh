# build -> all GPU tests -> bench -> rocprofv3 kernel trace of the bench; stops at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; exit 1; }
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_device.log 2>&1 || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_device.log; exit 1; }
tail -1 gpurun_out/bench_device.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r4 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_r4.log 2>&1 || { echo "prof failed rc=$?"; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_r4 -name "*.db" | head -1) 40 > gpurun_out/prof_r4_summary.md
echo ALL OK

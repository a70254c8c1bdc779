# round-4 start: full GPU suite (verbose, names each test), smoke, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4s_gpu.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/r4s_gpu.log; exit 1; }
tail -1 gpurun_out/r4s_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4s_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4s_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/r4s_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r4s_bench.log; exit 1; }
tail -1 gpurun_out/r4s_bench.log

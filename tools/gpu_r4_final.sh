# round-4 final: full GPU suite, smoke, bench, kernel trace of the headline (summaries -> profiles/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4f_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r4f_gpu.log
[ $rc -le 1 ] || exit 1  # (1: failures, reported above; anything else: stop)
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4f_smoke.log; exit 1; }
tail -1 gpurun_out/r4f_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r4f_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r4f_bench.log; exit 1; }
tail -1 gpurun_out/r4f_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4f_prof -o r4f -- python bench.py --steps 10 --warmup 3 > gpurun_out/r4f_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r4f_prof.log; exit 1; }
echo prof ok

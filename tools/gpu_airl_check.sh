set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/engine tests/ops tests/util tests/rewards tests/algorithms > gpurun_out/pytest_engine.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/pytest_engine.log; exit 1; }
tail -1 gpurun_out/pytest_engine.log
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 4 --warmup 1 --eval-episodes 0 > gpurun_out/airl_bench.log 2>&1 || { tail -20 gpurun_out/airl_bench.log; exit 1; }
grep config gpurun_out/airl_bench.log | cut -c1-200

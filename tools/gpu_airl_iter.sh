set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/engine/test_device_engine.py -x -q -m gpu -k "airl" --timeout 300 --timeout-method thread > gpurun_out/pytest_airl.log 2>&1 || { echo "airl tests failed"; tail -40 gpurun_out/pytest_airl.log; exit 1; }
tail -2 gpurun_out/pytest_airl.log
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 4 --warmup 1 --eval-episodes 0 > gpurun_out/airl_bench.log 2>&1 || { tail -20 gpurun_out/airl_bench.log; exit 1; }
grep config gpurun_out/airl_bench.log

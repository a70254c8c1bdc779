set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/algorithms/test_bc.py tests/engine/test_device_preference.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_bc.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_bc.log; exit 1; }
tail -3 gpurun_out/pytest_bc.log
timeout -k 10 300 python -u -m cProfile -o gpurun_out/dagger4.prof benchmarking/bench_configs.py --configs dagger_pong --steps 3 --warmup 1 --eval-episodes 0 > gpurun_out/dagger4.log 2>&1 || { echo "dagger failed"; tail -20 gpurun_out/dagger4.log; exit 1; }
tail -1 gpurun_out/dagger4.log
echo ALL OK

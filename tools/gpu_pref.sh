# device DRLHP agent: engine tests, then the preference config bench (+ cProfile)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/engine -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_engine.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_engine.log; exit 1; }
tail -3 gpurun_out/pytest_engine.log
timeout -k 10 300 python -u -m cProfile -o gpurun_out/pref2.prof benchmarking/bench_configs.py --configs preference_walker2d --steps 3 --warmup 1 --eval-episodes 2 > gpurun_out/pref2.log 2>&1 || { echo "pref failed"; tail -30 gpurun_out/pref2.log; exit 1; }
tail -2 gpurun_out/pref2.log
echo ALL OK

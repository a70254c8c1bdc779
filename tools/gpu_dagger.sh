set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/engine/test_device_dagger.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/dagger2.log 2>&1 || { tail -30 gpurun_out/dagger2.log; exit 1; }
tail -2 gpurun_out/dagger2.log
timeout -k 10 600 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 2 --warmup 1 --eval-episodes 0 > gpurun_out/dagger_bench.log 2>&1 || { tail -30 gpurun_out/dagger_bench.log; exit 1; }
grep config gpurun_out/dagger_bench.log

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-conv}
timeout -k 10 300 python -u -m pytest tests/ops/test_conv.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_conv_$TAG.log 2>&1 || { echo "conv tests failed rc=$?"; tail -40 gpurun_out/pytest_conv_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_conv_$TAG.log
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/conv_bench_$TAG.log 2>&1 || { echo "conv bench failed rc=$?"; tail -20 gpurun_out/conv_bench_$TAG.log; exit 1; }
cat gpurun_out/conv_bench_$TAG.log
echo ALL OK

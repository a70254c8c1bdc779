set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/ops/test_conv.py tests/ops/test_kernels.py -x -q -m gpu -k "conv or cnn or same_padding" --timeout 200 --timeout-method thread > gpurun_out/pytest_conv_iter.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_conv_iter.log; exit 1; }
tail -2 gpurun_out/pytest_conv_iter.log
timeout -k 10 300 python -u tools/reward_cnn_bench.py 2>&1 | grep -v Warn
timeout -k 10 300 python -u tools/conv_bench.py 2>&1 | grep -v Warn

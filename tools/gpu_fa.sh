set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/ops/test_fused_adam.py tests/algorithms/test_bc.py tests/engine/test_device_dagger.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/fa.log 2>&1 || { grep -E "Error|error|FAIL|assert" gpurun_out/fa.log | head -30; exit 1; }
tail -2 gpurun_out/fa.log
timeout -k 10 300 python -u tools/cnn_bc_probe.py 2>&1 | grep -v Warn
timeout -k 10 300 python -u tools/dagger_probe.py 2>&1 | grep -v Warn

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-eng}
timeout -k 10 500 python -u -m pytest tests/engine/test_device_engine.py -x -v -m gpu --timeout 200 --timeout-method thread ${KSEL:+-k "$KSEL"} > gpurun_out/pytest_engine_$TAG.log 2>&1 || { echo "engine tests failed rc=$?"; grep -v "^\s*$" gpurun_out/pytest_engine_$TAG.log | tail -40; exit 1; }
tail -3 gpurun_out/pytest_engine_$TAG.log

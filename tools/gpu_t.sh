# run selected GPU tests: bash tools/gpu_t.sh <pytest args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/pytest_sel.log 2>&1 || { echo "FAILED rc=$?"; grep -E "FAILED|Error|passed|failed|assert" gpurun_out/pytest_sel.log | tail -30; exit 1; }
tail -3 gpurun_out/pytest_sel.log

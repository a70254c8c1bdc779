set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ops > gpurun_out/pytest_ops.log 2>&1 || { echo "ops tests failed rc=$?"; tail -40 gpurun_out/pytest_ops.log; exit 1; }
tail -2 gpurun_out/pytest_ops.log
timeout -k 10 200 python -u tools/bc_step_probe.py > gpurun_out/bc_probe.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/bc_probe.log; exit 1; }
grep -v Warn gpurun_out/bc_probe.log | tail -2
timeout -k 10 300 python -u tools/bc_op_trace.py > gpurun_out/bc_ops.log 2>&1; echo rc=$?
grep -v Warn gpurun_out/bc_ops.log | tail -45 | cut -c1-60,100-190

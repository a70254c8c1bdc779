set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ops tests/algorithms/test_bc.py tests/algorithms/test_mce_irl.py tests/algorithms/test_density.py tests/engine/test_device_dagger.py tests/rl tests/data tests/algorithms/test_sqil.py tests/algorithms/test_dagger.py > gpurun_out/pytest_ops.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/pytest_ops.log; exit 1; }
tail -2 gpurun_out/pytest_ops.log
timeout -k 10 200 python -u tools/bc_step_probe.py > gpurun_out/bc_probe.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/bc_probe.log; exit 1; }
grep -v Warn gpurun_out/bc_probe.log | tail -1
timeout -k 10 400 python -u tools/dagger_probe.py > gpurun_out/dagger_probe.log 2>&1 || { echo "probe failed rc=$?"; tail -30 gpurun_out/dagger_probe.log; exit 1; }
grep -v Warn gpurun_out/dagger_probe.log | grep "round\|step\|replay"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bc -o run -- python3 $GRAFT_REPO_ROOT/tools/bc_step_probe.py > $GRAFT_REPO_ROOT/gpurun_out/prof_bc.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_bc.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_bc -name "*.db" | head -1) 60 > gpurun_out/prof_bc_summary.md
rm -rf gpurun_out/prof_bc
head -40 gpurun_out/prof_bc_summary.md | cut -c1-150

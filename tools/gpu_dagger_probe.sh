set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/engine/test_device_dagger.py > gpurun_out/pytest_dagger.log 2>&1 || { echo "dagger tests failed rc=$?"; tail -40 gpurun_out/pytest_dagger.log; exit 1; }
tail -1 gpurun_out/pytest_dagger.log
timeout -k 10 400 python -u tools/dagger_probe.py > gpurun_out/dagger_probe.log 2>&1 || { echo "probe failed rc=$?"; tail -30 gpurun_out/dagger_probe.log; exit 1; }
grep -v Warn gpurun_out/dagger_probe.log | grep "round\|step\|replay"

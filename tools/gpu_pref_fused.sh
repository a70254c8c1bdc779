# fused preference minibatch: tests + DRLHP probe (fused on / off)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/engine/test_device_preference.py > gpurun_out/pytest_pref.log 2>&1 || { echo "FAILED rc=$?"; grep -E "FAILED|Error|passed|failed|assert" gpurun_out/pytest_pref.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest_pref.log
timeout -k 10 600 python -u tools/pref_probe.py > gpurun_out/pref_probe_fused.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/pref_probe_fused.log; exit 1; }
grep -v Warn gpurun_out/pref_probe_fused.log | grep "iteration\|rollout"
IMITATION_AMD_PREF_FUSED=0 timeout -k 10 600 python -u tools/pref_probe.py > gpurun_out/pref_probe_unfused.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/pref_probe_unfused.log; exit 1; }
grep -v Warn gpurun_out/pref_probe_unfused.log | grep "iteration\|rollout"

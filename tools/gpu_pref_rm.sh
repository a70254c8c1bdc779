set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/engine/test_device_preference.py > gpurun_out/pytest_pref.log 2>&1 || { echo "FAILED rc=$?"; grep -E "FAILED|Error|passed|failed|assert" gpurun_out/pytest_pref.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_pref.log
timeout -k 10 300 python tools/pref_rm_probe.py > gpurun_out/pref_rm.log 2>&1 && grep "reward training" gpurun_out/pref_rm.log &&
IMITATION_AMD_PREF_EPOCH_GRAPH=0 timeout -k 10 300 python tools/pref_rm_probe.py > gpurun_out/pref_rm1.log 2>&1 && grep "reward training" gpurun_out/pref_rm1.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pref_rm -o run -- python tools/pref_rm_probe.py 500 100 50 > gpurun_out/prof_pref_rm.log 2>&1 && echo PROF_OK

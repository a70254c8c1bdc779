set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/pref_probe.py > gpurun_out/pref_probe.log 2>&1 || { echo "probe failed rc=$?"; tail -30 gpurun_out/pref_probe.log; exit 1; }
grep -v Warn gpurun_out/pref_probe.log | grep "iteration\|rollout"

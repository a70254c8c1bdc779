set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/pref_ppo_probe.py > gpurun_out/pref_ppo.log 2>&1 || { echo "probe failed rc=$?"; tail -30 gpurun_out/pref_ppo.log; exit 1; }
grep rc_gmax gpurun_out/pref_ppo.log

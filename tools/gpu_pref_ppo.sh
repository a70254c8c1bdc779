set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for R in ${RECIPES:-preference_walker2d}; do
  RECIPE=$R timeout -k 10 300 python -u tools/pref_ppo_probe.py > gpurun_out/ppo_gmax_$R.log 2>&1 || { echo "probe $R failed rc=$?"; tail -30 gpurun_out/ppo_gmax_$R.log; exit 1; }
  echo $R; grep rc_gmax gpurun_out/ppo_gmax_$R.log
done

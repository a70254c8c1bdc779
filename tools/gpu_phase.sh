set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ppo_phase_probe.py > gpurun_out/phase_probe.log 2>&1 && timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/scale_probe.log 2>&1; echo rc=$?
grep -v Warn gpurun_out/phase_probe.log; grep -v Warn gpurun_out/scale_probe.log

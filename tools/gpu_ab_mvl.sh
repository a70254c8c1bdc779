set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
(rocm-smi --showclocks > gpurun_out/clocks.log 2>&1 || true)
IA_PPO_MVL=0 timeout -k 10 300 python -u tools/ppo_phase_probe.py > gpurun_out/phase_nomvl.log 2>&1 && timeout -k 10 300 python -u tools/ppo_phase_probe.py > gpurun_out/phase_mvl.log 2>&1; echo rc=$?
grep -v Warn gpurun_out/phase_nomvl.log | grep -v amdgpu.ids; grep -v Warn gpurun_out/phase_mvl.log | grep -v amdgpu.ids
grep -i "sclk\|mclk" gpurun_out/clocks.log | head -4

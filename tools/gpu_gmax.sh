# AIRL emulated W=4/8: cooperating-workgroup cap 64 (default) vs 32 / 16 (more chunks per workgroup)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for gm in 0 32 16; do
  RC_GMAX=$gm WS=4,8 CONFIG=airl timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/gmax_$gm.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/gmax_$gm.log; exit 1; }
  echo "gmax=$gm"; grep "xchg2=1: ppo update" gpurun_out/gmax_$gm.log
done

# round-end rehearsal: full GPU test suite, smoke, 1-GPU headline bench, every benchmark config
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_full.sh || exit 1
CFGS=${CFGS:-all} STEPS=${STEPS:-2} bash tools/gpu_configs.sh ${TAG:-round} || exit 1

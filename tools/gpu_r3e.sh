# end-of-session measurements: headline trace + SQ counters, all config lines, full GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_bench_prof.sh || exit 1
CFGS=all STEPS=2 timeout -k 10 900 bash tools/gpu_configs.sh r3e || exit 1

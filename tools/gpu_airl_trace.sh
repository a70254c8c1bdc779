# kernel trace of the AIRL-Hopper config (3 rounds)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_airl -o run -- python $GRAFT_REPO_ROOT/benchmarking/bench_configs.py --configs airl_hopper --steps 3 --warmup 1 --eval-episodes 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_airl.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_airl.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_airl -name "*.db" | head -1) 40 > gpurun_out/prof_airl_summary.md
rm -rf gpurun_out/prof_airl
grep config gpurun_out/prof_airl.log | cut -c1-200
head -24 gpurun_out/prof_airl_summary.md

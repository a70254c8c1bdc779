# AIRL-Hopper round timeline (rocprofv3 kernel trace of bench_configs, one round listed)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_airl -o run -- python3 $GRAFT_REPO_ROOT/benchmarking/bench_configs.py --configs airl_hopper --steps 6 --warmup 1 --eval-episodes 0 --out /tmp/airl_tl.jsonl > $GRAFT_REPO_ROOT/gpurun_out/prof_airl.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_airl.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_airl -name "*.db" | head -1) 25 > gpurun_out/prof_airl_summary.md
python tools/prof_timeline.py $(find gpurun_out/prof_airl -name "*.db" | head -1) rollout_chain_kernel 4 > gpurun_out/prof_airl_timeline.md
rm -rf gpurun_out/prof_airl
head -20 gpurun_out/prof_airl_summary.md

# kernel trace of the DRLHP-Walker config (reference seals_walker settings), 1 GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_pref -o run -- python $GRAFT_REPO_ROOT/benchmarking/bench_configs.py --configs preference_walker2d --steps 2 --warmup 1 --eval-episodes 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_pref.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_pref.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_pref -name "*.db" | head -1) 30 > gpurun_out/prof_pref_summary.md
rm -rf gpurun_out/prof_pref
grep '"config"' gpurun_out/prof_pref.log | cut -c1-220
head -20 gpurun_out/prof_pref_summary.md

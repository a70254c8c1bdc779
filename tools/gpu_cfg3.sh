# all BASELINE configs on one GPU + kernel trace of the DRLHP config
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u benchmarking/bench_configs.py --configs all --steps 3 --warmup 1 --out gpurun_out/cfg3.jsonl > gpurun_out/cfg3.log 2>&1 || { echo "cfg failed rc=$?"; tail -30 gpurun_out/cfg3.log; exit 1; }
cat gpurun_out/cfg3.jsonl
timeout -k 10 300 python -u -m cProfile -o gpurun_out/dagger3.prof benchmarking/bench_configs.py --configs dagger_pong --steps 2 --warmup 1 --eval-episodes 0 > gpurun_out/dagger3.log 2>&1 || { echo "dagger prof failed"; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_pref -o run -- python $GRAFT_REPO_ROOT/benchmarking/bench_configs.py --configs preference_walker2d --steps 2 --warmup 1 --eval-episodes 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_pref.log 2>&1 || { echo "prof failed rc=$?"; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_pref -name "*.db" | head -1) 30 > gpurun_out/prof_pref_summary.md
echo ALL OK

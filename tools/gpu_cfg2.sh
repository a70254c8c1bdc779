# all BASELINE configs on one GPU + cProfile of the slow host-driven ones
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u benchmarking/bench_configs.py --configs all --steps 3 --warmup 1 --out gpurun_out/cfg_all.jsonl > gpurun_out/cfg_all.log 2>&1 || { echo "cfg failed rc=$?"; tail -30 gpurun_out/cfg_all.log; exit 1; }
cat gpurun_out/cfg_all.jsonl
timeout -k 10 300 python -u -m cProfile -o gpurun_out/dagger.prof benchmarking/bench_configs.py --configs dagger_pong --steps 2 --warmup 1 --eval-episodes 0 > gpurun_out/dagger_prof.log 2>&1 || { echo "dagger prof failed"; exit 1; }
timeout -k 10 300 python -u -m cProfile -o gpurun_out/pref.prof benchmarking/bench_configs.py --configs preference_walker2d --steps 2 --warmup 1 --eval-episodes 0 > gpurun_out/pref_prof.log 2>&1 || { echo "pref prof failed"; exit 1; }
echo ALL OK

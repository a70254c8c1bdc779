# round-4: kernel trace of DAgger-Pong rounds (device collector + epoch-graph BC)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4e_prof -o r4e -- python -u benchmarking/bench_configs.py --configs dagger_pong --steps 2 --warmup 1 --eval-episodes 1 > gpurun_out/r4e_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r4e_prof.log; exit 1; }
grep config gpurun_out/r4e_prof.log | cut -c1-300

# fused AIRL discriminator: tests + AIRL bench config
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/engine/test_device_engine.py -x -v -m gpu -k "airl" --timeout 300 --timeout-method thread > gpurun_out/pytest_airl.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|passed|failed|assert|Mismatch|Greatest" gpurun_out/pytest_airl.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_airl.log
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 3 --warmup 1 > gpurun_out/bench_airl.log 2>&1 || { echo "airl bench failed"; tail -20 gpurun_out/bench_airl.log; exit 1; }
grep "{" gpurun_out/bench_airl.log | tail -2
mkdir -p gpurun_out/prof_airl2
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_airl2 -o run -- python3 $GRAFT_REPO_ROOT/benchmarking/bench_configs.py --configs airl_hopper --steps 3 --warmup 1 --eval-episodes 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_airl2.log 2>&1 || { echo "prof failed"; exit 1; }
echo ALL OK

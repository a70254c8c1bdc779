# multi-workgroup RunningNorm: numerics tests, device-engine tests, AIRL-Hopper config
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/util/test_networks.py tests/engine/test_device_engine.py tests/parallel/test_oneshot.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/norm_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|passed|failed" gpurun_out/norm_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/norm_tests.log
timeout -k 10 300 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 3 --warmup 1 --eval-episodes 2 > gpurun_out/airl_norm.log 2>&1 || { tail -20 gpurun_out/airl_norm.log; exit 1; }
grep '"config"' gpurun_out/airl_norm.log | cut -c1-250

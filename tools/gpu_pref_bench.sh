set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/engine/test_device_preference.py tests/ops/test_fused_adam.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pref_t.log 2>&1 || { grep -E "Error|error|FAIL|assert" gpurun_out/pref_t.log | head -30; exit 1; }
tail -1 gpurun_out/pref_t.log
timeout -k 10 900 python -u benchmarking/bench_configs.py --configs preference_walker2d --steps ${STEPS:-2} --warmup 1 --eval-episodes 0 > gpurun_out/pref_bench.log 2>&1 || { tail -30 gpurun_out/pref_bench.log; exit 1; }
grep -E "config|Query" gpurun_out/pref_bench.log

# round-4 session: new GPU tests (exchange levels, AIRL split rounds) + AIRL config timing + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/engine/test_device_engine.py -k "exchange_levels or airl_pipelined or ppo_kernel" > gpurun_out/r4b_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4b_tests.log; exit 1; }
tail -2 gpurun_out/r4b_tests.log
for split in 0 1; do
  IMITATION_AMD_AIRL_SPLIT=$split timeout -k 10 400 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 3 --warmup 1 --eval-episodes 2 --out gpurun_out/r4b_airl_s$split.jsonl > gpurun_out/r4b_airl_s$split.log 2>&1 || { echo "airl bench failed"; tail -30 gpurun_out/r4b_airl_s$split.log; exit 1; }
  echo "split=$split"; cut -c1-300 gpurun_out/r4b_airl_s$split.jsonl
done
VARIANTS="geo4 geo5" WS=1,8 bash tools/gpu_r4_ab.sh

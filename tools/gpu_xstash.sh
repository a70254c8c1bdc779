# item-split first-level exchange (G > 16): PPO device tests + AIRL scale probe W=1..8 (bitwise check vs one-level)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/engine/test_device_engine.py -m gpu -k "ppo" > gpurun_out/xstash_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/xstash_tests.log; exit 1; }
tail -2 gpurun_out/xstash_tests.log
for c in ${CONFIGS:-airl}; do
  CONFIG=$c timeout -k 10 400 python -u tools/ppo_scale_probe.py > gpurun_out/xstash_probe_$c.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/xstash_probe_$c.log; exit 1; }
  echo "$c"; grep "ppo update\|cycles" gpurun_out/xstash_probe_$c.log
done

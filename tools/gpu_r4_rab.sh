# round-4: A/B of rollout-chain builds (ab/<variant>.so): chain timing (GAIL / AIRL recipes) + headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SO=$(ls imitation_amd/_C.cpython-*.so)
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/engine/test_device_engine.py -k "rollout or rounds or pipelined" > gpurun_out/rab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/rab_tests.log; exit 1; }
tail -1 gpurun_out/rab_tests.log
cp $SO /tmp/orig.so
for rep in 1 2; do
for v in ${VARIANTS}; do
  cp ab/$v.so $SO
  for r in gail_halfcheetah airl_hopper; do
    RECIPE=$r timeout -k 10 200 python -u tools/rollout_probe.py > gpurun_out/rab_${v}_$r.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/rab_${v}_$r.log; cp /tmp/orig.so $SO; exit 1; }
    echo "$v $r $(grep chain gpurun_out/rab_${v}_$r.log)"
  done
  timeout -k 10 200 python bench.py > gpurun_out/rab_${v}_bench.log 2>&1 || { echo "bench failed"; cp /tmp/orig.so $SO; exit 1; }
  echo "$v bench $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rab_${v}_bench.log)"
done
done
cp /tmp/orig.so $SO

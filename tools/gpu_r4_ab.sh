# round-4 A/B of PPO kernel builds on one box: ab/<variant>.so swapped in for the probe + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SO=$(ls imitation_amd/_C.cpython-*.so)
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/engine/test_device_engine.py -k "ppo_kernel" > gpurun_out/ab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ab_tests.log
[ $rc -le 1 ] || exit 1  # (1: test failures, still measured; anything else: stop)
cp $SO /tmp/orig.so
for v in ${VARIANTS:-pre head fix}; do
  cp ab/$v.so $SO
  for c in gail airl drlhp; do
    ws=${WS:-1}; [ $c = drlhp ] && ws=1
    CONFIG=$c WS=$ws timeout -k 10 200 python -u tools/ppo_scale_probe.py > gpurun_out/ab_${v}_$c.log 2>&1 || { echo "$v $c probe failed"; tail -20 gpurun_out/ab_${v}_$c.log; cp /tmp/orig.so $SO; exit 1; }
    echo "== $v"; grep -v Warn gpurun_out/ab_${v}_$c.log | grep -v amdgpu.ids
  done
  timeout -k 10 200 python -u bench.py > gpurun_out/ab_${v}_bench.log 2>&1 || { echo "$v bench failed"; tail -20 gpurun_out/ab_${v}_bench.log; cp /tmp/orig.so $SO; exit 1; }
  echo "== $v bench"; grep metric gpurun_out/ab_${v}_bench.log | cut -c1-260
done
cp /tmp/orig.so $SO

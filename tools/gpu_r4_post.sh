# round-4: rollout_post_kernel A/B (ab/<variant>.so): engine tests on the in-tree build, then per
# variant the post-kernel time from a kernel trace (GAIL bench, AIRL config) and a plain bench run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SO=$(ls imitation_amd/_C.cpython-*.so)
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/engine/test_device_engine.py > gpurun_out/post_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/post_tests.log; exit 1; }
tail -1 gpurun_out/post_tests.log
cp $SO /tmp/orig.so
for v in ${VARIANTS}; do
  cp ab/$v.so $SO
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/post_${v}_g -o p -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/post_${v}_g.log 2>&1 || { echo "$v gail trace failed"; tail -20 gpurun_out/post_${v}_g.log; cp /tmp/orig.so $SO; exit 1; }
  echo "$v gail $(python3 tools/prof_summary.py $(ls gpurun_out/post_${v}_g/*.db | head -1) 40 | grep -E "${KGREP:-rollout_post}")"
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/post_${v}_a -o p -- python3 benchmarking/bench_configs.py --configs airl_hopper --steps 3 --warmup 1 --eval-episodes 1 > gpurun_out/post_${v}_a.log 2>&1 || { echo "$v airl trace failed"; tail -20 gpurun_out/post_${v}_a.log; cp /tmp/orig.so $SO; exit 1; }
  echo "$v airl $(python3 tools/prof_summary.py $(ls gpurun_out/post_${v}_a/*.db | head -1) 60 | grep -E "${KGREP:-rollout_post}")"
  timeout -k 10 200 python bench.py > gpurun_out/post_${v}_bench.log 2>&1 || { echo "$v bench failed"; cp /tmp/orig.so $SO; exit 1; }
  echo "$v bench $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/post_${v}_bench.log)"
done
cp /tmp/orig.so $SO

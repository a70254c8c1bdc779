# round-4: engine + algorithm GPU tests on the in-tree build, then bench / AIRL config A/B of ab/<variant>.so
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SO=$(ls imitation_amd/_C.cpython-*.so)
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/engine tests/algorithms > gpurun_out/nc_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/nc_tests.log; exit 1; }
tail -1 gpurun_out/nc_tests.log
cp $SO /tmp/orig.so
for rep in 1 2; do
for v in ${VARIANTS}; do
  cp ab/$v.so $SO
  timeout -k 10 200 python bench.py > gpurun_out/nc_${v}_bench.log 2>&1 || { echo "$v bench failed"; tail -20 gpurun_out/nc_${v}_bench.log; cp /tmp/orig.so $SO; exit 1; }
  echo "$v bench $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/nc_${v}_bench.log)"
  timeout -k 10 300 python -u benchmarking/bench_configs.py --configs airl_hopper --steps 4 --warmup 1 --eval-episodes 1 --out gpurun_out/nc_${v}_airl.jsonl > gpurun_out/nc_${v}_airl.log 2>&1 || { echo "$v airl failed"; tail -20 gpurun_out/nc_${v}_airl.log; cp /tmp/orig.so $SO; exit 1; }
  echo "$v airl $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/nc_${v}_airl.jsonl | tail -1)"
done
done
cp /tmp/orig.so $SO

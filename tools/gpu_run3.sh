# build -> engine GPU tests -> phase profile -> bench; stops at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; exit 1; }
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_engine.log 2>&1 || { echo "pytest failed rc=$?"; exit 1; }
timeout -k 10 300 python tools/rollout_prof.py > gpurun_out/rollout_prof.log 2>&1 || { echo "prof failed rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --engine device --steps 10 --warmup 2 > gpurun_out/bench_device.log 2>&1 || { echo "bench failed rc=$?"; exit 1; }
echo ALL OK

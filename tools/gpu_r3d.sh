# BC head loads-in-flight + XCD default: BC tests / trace, engine tests, DAgger line, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/algorithms/test_bc.py tests/engine/test_device_engine.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r3d.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAILED|Error|error|passed|failed" gpurun_out/pytest_r3d.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r3d.log
bash tools/gpu_bc_prof.sh | head -14
CFGS=dagger_pong STEPS=2 timeout -k 10 600 bash tools/gpu_configs.sh r3d
timeout -k 10 300 python bench.py > gpurun_out/bench_r3d.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_r3d.log; exit 1; }
tail -1 gpurun_out/bench_r3d.log

# round-4: new fail-fast tests, full GPU suite, smoke, bench, kernel trace of the headline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/engine/test_device_engine.py tests/engine/test_device_dagger.py tests/algorithms/test_bc.py tests/parallel/test_oneshot.py -m gpu -k "timeout_raises or ppo_kernel_matches or epoch_graph or pipelined or agent_gather or dp_fused_bc" > gpurun_out/r4a_new.log 2>&1 || { echo "new tests failed"; tail -40 gpurun_out/r4a_new.log; exit 1; }
tail -1 gpurun_out/r4a_new.log
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4a_gpu.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/r4a_gpu.log; exit 1; }
tail -1 gpurun_out/r4a_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4a_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/r4a_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r4a_bench.log; exit 1; }
tail -1 gpurun_out/r4a_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4a_prof -o r4a -- python bench.py --steps 10 --warmup 3 > gpurun_out/r4a_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r4a_prof.log; exit 1; }
echo prof ok
CONFIG=gail WS=1,8 timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/r4p_gail.log 2>&1 || { echo "gail probe failed"; tail -20 gpurun_out/r4p_gail.log; exit 1; }
cat gpurun_out/r4p_gail.log | grep -v Warn
CONFIG=airl WS=1,8 timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/r4p_airl.log 2>&1 || { echo "airl probe failed"; tail -20 gpurun_out/r4p_airl.log; exit 1; }
cat gpurun_out/r4p_airl.log | grep -v Warn
CONFIG=drlhp WS=1 timeout -k 10 300 python -u tools/ppo_scale_probe.py > gpurun_out/r4p_drlhp.log 2>&1 || { echo "drlhp probe failed"; tail -20 gpurun_out/r4p_drlhp.log; exit 1; }
cat gpurun_out/r4p_drlhp.log | grep -v Warn

# round-4: DAgger paired-head collector: tests + DAgger-Pong config + probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/engine/test_device_dagger.py > gpurun_out/r4h_tests.log 2>&1 || { echo "dagger tests failed"; tail -30 gpurun_out/r4h_tests.log; exit 1; }
tail -1 gpurun_out/r4h_tests.log
timeout -k 10 300 python -u tools/dagger_probe.py > gpurun_out/r4h_dagger.log 2>&1 || { echo "dagger probe failed"; tail -30 gpurun_out/r4h_dagger.log; exit 1; }
grep "round \|train step\|chunk replay" gpurun_out/r4h_dagger.log
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 3 --warmup 1 --eval-episodes 2 --out gpurun_out/r4h_dagger.jsonl > gpurun_out/r4h_cfg.log 2>&1 || { echo "dagger config failed"; tail -30 gpurun_out/r4h_cfg.log; exit 1; }
cut -c1-300 gpurun_out/r4h_dagger.jsonl

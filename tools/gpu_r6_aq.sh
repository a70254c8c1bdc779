#!/bin/bash
# round 6 call AQ: the final tree (after the Adam zeroing change) -- whole GPU suite + smoke, headline bench, DAgger reference schedule
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6aq_gpu_suite.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6aq_smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > gpurun_out/r6aq_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 --out gpurun_out/r6aq_dagger.jsonl > gpurun_out/r6aq_dagger.log 2>&1

#!/bin/bash
# round 6 call AI: final tree -- the whole GPU suite + smoke (as the driver runs them), then the headline bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6ai_gpu_suite.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6ai_smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > gpurun_out/r6ai_bench.log 2>&1

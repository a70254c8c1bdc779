#!/bin/bash
# round 5, call AP (final, end of round, after the last DAgger knobs): full GPU suite + smoke + headline bench + every bench config at HEAD
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_ap_gpu_suite.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_ap_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r5_ap_bench.log 2>&1 &&
timeout -k 10 900 python -u benchmarking/bench_configs.py --out gpurun_out/r5_ap_bench_configs.jsonl > gpurun_out/r5_ap_bench_configs.log 2>&1 &&
timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 > gpurun_out/r5_ap_dagger.log 2>&1

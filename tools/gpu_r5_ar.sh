#!/bin/bash
# round 5, call AR: bench_configs with the per-config default timed steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u benchmarking/bench_configs.py --out gpurun_out/r5_ar_bench_configs.jsonl > gpurun_out/r5_ar_bench_configs.log 2>&1

#!/bin/bash
# round 6 call AB: end-of-round numbers -- headline bench twice, all bench configs (DAgger reference schedule,
# AIRL, DRLHP, ...), kernel trace of the headline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u bench.py > gpurun_out/r6ab_bench.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py >> gpurun_out/r6ab_bench.log 2>&1 || exit $?
timeout -k 10 700 python -u benchmarking/bench_configs.py --configs all --out gpurun_out/r6ab_configs.jsonl \
  > gpurun_out/r6ab_configs.log 2>&1 || exit $?
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r6_ab_kt -o run -- python3 $R/bench.py --steps 20 --warmup 3 --eval-episodes 0 > $R/gpurun_out/r6ab_kt.log 2>&1 || exit $?
cd $R && cp $(find /tmp/r6_ab_kt -name "*kernel_stats.csv" | head -1) gpurun_out/r6ab_kernel_stats.csv && rm -rf /tmp/r6_ab_kt

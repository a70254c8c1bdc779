#!/bin/bash
# round 6 call B: bench with the expert in a child process (cold then warm), in-process slowdown probe
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 400 python -u bench.py > gpurun_out/r6b_bench_cold.log 2>&1 || exit $?
t1=$(date +%s)
timeout -k 10 400 python -u bench.py > gpurun_out/r6b_bench_warm.log 2>&1 || exit $?
t2=$(date +%s)
echo "cold $((t1 - t0)) s, warm $((t2 - t1)) s" > gpurun_out/r6b_times.txt
timeout -k 10 400 python -u tools/expert_inproc_probe.py > gpurun_out/r6b_probe.log 2>&1 || exit $?

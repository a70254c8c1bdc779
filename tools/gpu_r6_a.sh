#!/bin/bash
# round 6 call A: bench.py with the imitation-quality phase (cold, then cached expert)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
s=$(date +%s.%N)
timeout -k 10 400 python -u bench.py > gpurun_out/r6a_bench_cold.log 2>&1 || exit $?
e=$(date +%s.%N); echo "cold wall $(echo "$e - $s" | bc)" | tee -a gpurun_out/r6a_times.txt
s=$(date +%s.%N)
timeout -k 10 400 python -u bench.py > gpurun_out/r6a_bench_warm.log 2>&1 || exit $?
e=$(date +%s.%N); echo "warm wall $(echo "$e - $s" | bc)" | tee -a gpurun_out/r6a_times.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_contract.py -m gpu > gpurun_out/r6a_test.log 2>&1 || exit $?
tail -2 gpurun_out/r6a_bench_cold.log gpurun_out/r6a_bench_warm.log

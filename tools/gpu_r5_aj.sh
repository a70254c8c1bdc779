#!/bin/bash
# round 5, call AJ: DAgger BC-statistics twin on a high-priority stream (and with pair + wait relaunches): A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/engine/test_device_dagger.py -m gpu -k "async or growing" > gpurun_out/r5_aj_tests.log 2>&1 &&
for v in base prio priopw base prio priopw; do
  case $v in
    base) export IMITATION_AMD_DAGGER_STATS_PRIORITY=0 IMITATION_AMD_BC_GRAPH_WAIT=0 IMITATION_AMD_BC_GRAPH_PAIR=0;;
    prio) export IMITATION_AMD_DAGGER_STATS_PRIORITY=1 IMITATION_AMD_BC_GRAPH_WAIT=0 IMITATION_AMD_BC_GRAPH_PAIR=0;;
    priopw) export IMITATION_AMD_DAGGER_STATS_PRIORITY=1 IMITATION_AMD_BC_GRAPH_WAIT=1 IMITATION_AMD_BC_GRAPH_PAIR=1;;
  esac
  timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 > gpurun_out/r5_aj_$v.log 2>&1 || exit 1
  grep '"value"' gpurun_out/r5_aj_$v.log | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/r5_aj_ab.jsonl
  echo "$v done"
done

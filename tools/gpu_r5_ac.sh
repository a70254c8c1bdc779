#!/bin/bash
# round 5, call AC: BC epoch graph relaunch -- wait on the previous launch's event (outside hipGraphLaunch),
# one or two instances per size. Bitwise tests, then an interleaved DAgger-Pong A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/engine/test_device_dagger.py -m gpu > gpurun_out/r5_ac_tests.log 2>&1 &&
for v in base wait pairwait base wait pairwait; do
  case $v in
    base) export IMITATION_AMD_BC_GRAPH_WAIT=0 IMITATION_AMD_BC_GRAPH_PAIR=0;;
    wait) export IMITATION_AMD_BC_GRAPH_WAIT=1 IMITATION_AMD_BC_GRAPH_PAIR=0;;
    pairwait) export IMITATION_AMD_BC_GRAPH_WAIT=1 IMITATION_AMD_BC_GRAPH_PAIR=1;;
  esac
  timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 > gpurun_out/r5_ac_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/r5_ac_$v.log | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/r5_ac_ab.jsonl
  echo "$v done"
done

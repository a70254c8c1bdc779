#!/bin/bash
# round 5, call W: DRLHP reward epochs launched eagerly for short schedules (no per-iteration capture)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/algorithms/test_preference_comparisons.py tests/engine -m gpu -k "pref or reward" > gpurun_out/r5_w_tests.log 2>&1 &&
IMITATION_AMD_PREF_EPOCH_GRAPH_MIN=1 timeout -k 10 600 python -u tools/pref_breakdown.py --iters 3 > gpurun_out/r5_w_pref_graph.log 2>&1 &&
timeout -k 10 600 python -u tools/pref_breakdown.py --iters 3 > gpurun_out/r5_w_pref_eager.log 2>&1

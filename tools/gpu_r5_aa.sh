#!/bin/bash
# round 5, call AA: training loops keep the pre-loop heap out of full GC passes (utils/gcfreeze.py): DRLHP A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in 1 0 1 0; do
  IMITATION_AMD_GC_FREEZE=$m timeout -k 10 400 python -u tools/pref_breakdown.py --iters 5 > gpurun_out/r5_aa_pref_g$m.log 2>&1 || exit 1
  tail -1 gpurun_out/r5_aa_pref_g$m.log | sed "s/^{/{\"gc_freeze\": $m, /" >> gpurun_out/r5_aa_ab.jsonl
  echo "freeze=$m done"
done &&
timeout -k 10 400 python -u benchmarking/bench_configs.py --configs preference_walker2d,dagger_pong --steps 4 --warmup 1 > gpurun_out/r5_aa_bench.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r5_aa_headline.log 2>&1

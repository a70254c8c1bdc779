#!/bin/bash
# round 5, call AO: DAgger statistics twin steps the learner alone (no paired expert forward): tests + A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/engine/test_device_dagger.py tests/algorithms/test_dagger.py -m gpu > gpurun_out/r5_ao_tests.log 2>&1 &&
for v in 1 0 1 0 1 0; do
  IMITATION_AMD_DAGGER_TWIN_LEARNER_ONLY=$v timeout -k 10 400 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 > gpurun_out/r5_ao_t$v.log 2>&1 || exit 1
  grep '"value"' gpurun_out/r5_ao_t$v.log | sed "s/^{/{\"learner_only\": $v, /" >> gpurun_out/r5_ao_ab.jsonl
  echo "learner_only=$v done"
done

#!/bin/bash
# round 6 call P: A/B of the conv weight-gradient block cap for BC-size layers (partial floats 1M / 2M / 4M:
# more blocks, more partial traffic), BC step + DAgger reference schedule per variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SO=imitation_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/orig.so
for v in cap1m cap2m cap4m cap1m; do
  cp ab/$v.so $SO
  echo "== $v" >> gpurun_out/r6p_bcstep.log
  timeout -k 10 120 python -u tools/bc_step_probe.py >> gpurun_out/r6p_bcstep.log 2>&1 || { cp /tmp/orig.so $SO; exit 1; }
done
for v in cap1m cap2m; do
  cp ab/$v.so $SO
  timeout -k 10 300 python -u benchmarking/bench_configs.py --configs dagger_pong --steps 4 --warmup 1 --out gpurun_out/r6p_dagger_$v.jsonl > gpurun_out/r6p_dagger_$v.log 2>&1 || { cp /tmp/orig.so $SO; exit 1; }
done
cp /tmp/orig.so $SO

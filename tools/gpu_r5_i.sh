#!/bin/bash
# round 5, call I: where a DAgger-Pong round's time goes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 4 --warmup 1 > gpurun_out/r5_i_dagger.log 2>&1 &&
timeout -k 10 400 python -u tools/dagger_breakdown.py --rounds 3 --warmup 1 --profile > gpurun_out/r5_i_dagger_prof.log 2>&1

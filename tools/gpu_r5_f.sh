#!/bin/bash
# round 5, call F: CLI path speed vs bench, expert-mode imitation on the synthetic locomotion envs
set -o pipefail
mkdir -p gpurun_out
export OUT=gpurun_out/r5_loco_quality.jsonl
rm -f $OUT
timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 > gpurun_out/r5_f_bench.log 2>&1 &&
timeout -k 10 300 python -u tools/cli_speed.py --rounds 60 --ckpt 10 > gpurun_out/r5_f_cli.log 2>&1 &&
timeout -k 10 300 python -u tools/cli_speed.py --rounds 60 --ckpt 10 --sync-logs > gpurun_out/r5_f_cli_sync.log 2>&1 &&
timeout -k 10 300 python -u tools/cli_speed.py --rounds 60 --ckpt 10 --no-pipeline > gpurun_out/r5_f_cli_nopipe.log 2>&1 &&
timeout -k 10 900 python -u tools/quality_probe.py gail:halfcheetah:5000000:5000000:0 airl:hopper:5000000:5000000:0 > gpurun_out/r5_f_loco.log 2>&1

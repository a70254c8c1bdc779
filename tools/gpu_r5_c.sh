#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/quality_sweep.py gail:12:512:8:0 gail:60:512:8:0 gail:12:16384:8:0 gail:60:16384:8:0 gail:12:512:32:0 airl:12:512:16:0 airl:60:512:16:0 airl:60:16384:16:0 > gpurun_out/r5_sweep.log 2>&1

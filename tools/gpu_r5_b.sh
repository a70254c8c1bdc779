#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/quality_diag.py gt device host > gpurun_out/r5_diag.log 2>&1

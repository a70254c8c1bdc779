#!/bin/bash
# round 5, call AT: PMC pass (SQ counters only, with --kernel-trace) over the DAgger-Pong round
# summarised per kernel on the box (top 24)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d /tmp/r5_at_pmc -o run -- python3 $R/tools/dagger_breakdown.py --rounds 1 > $R/gpurun_out/r5_at_pmc.log 2>&1 &&
cd $R && timeout -k 10 120 python3 tools/pmc_summary.py $(find /tmp/r5_at_pmc -name "*counter_collection.csv" | head -1) 24 > gpurun_out/r5_at_pmc.md 2>&1
rc=$?
rm -rf /tmp/r5_at_pmc
exit $rc

#!/bin/bash
# round 5, call AS: end-of-round PMC pass (SQ counters only, with --kernel-trace; no other trace domains)
# over the headline bench, summarised per kernel on the box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d /tmp/r5_as_pmc -o run -- python3 $R/bench.py --steps 4 --warmup 2 --eval-episodes 0 > $R/gpurun_out/r5_as_pmc.log 2>&1 &&
cd $R && timeout -k 10 120 python3 tools/pmc_summary.py $(find /tmp/r5_as_pmc -name "*counter_collection.csv" | head -1) 14 > gpurun_out/r5_as_pmc.md 2>&1
rc=$?
rm -rf /tmp/r5_as_pmc
exit $rc

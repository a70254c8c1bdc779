#!/bin/bash
# round 6 call O: end-of-round PMC pass (SQ counters only, with --kernel-trace; no other trace domains) and a
# kernel-trace --stats pass over the headline bench (no expert child / quality phase: --eval-episodes 0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d /tmp/r6_o_pmc -o run -- python3 $R/bench.py --steps 4 --warmup 2 --eval-episodes 0 > $R/gpurun_out/r6o_pmc.log 2>&1 &&
cd $R && timeout -k 10 120 python3 tools/pmc_summary.py $(find /tmp/r6_o_pmc -name "*counter_collection.csv" | head -1) 14 > gpurun_out/r6o_pmc.md 2>&1 || exit $?
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r6_o_kt -o run -- python3 $R/bench.py --steps 20 --warmup 3 --eval-episodes 0 > $R/gpurun_out/r6o_kt.log 2>&1 || exit $?
cd $R && cp $(find /tmp/r6_o_kt -name "*kernel_stats.csv" | head -1) gpurun_out/r6o_kernel_stats.csv
rm -rf /tmp/r6_o_pmc /tmp/r6_o_kt

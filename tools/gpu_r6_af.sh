#!/bin/bash
# round 6 call AF: PMC pass (SQ counters) over the fused BC step probe -- per-kernel VALU / MFMA / LDS / VMEM
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d /tmp/r6_af_pmc -o run -- python3 $R/tools/bc_step_probe.py > $R/gpurun_out/r6af_pmc.log 2>&1 &&
cd $R && timeout -k 10 120 python3 tools/pmc_summary.py $(find /tmp/r6_af_pmc -name "*counter_collection.csv" | head -1) 16 > gpurun_out/r6af_pmc.md 2>&1 || exit $?
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-trace --output-format csv -d /tmp/r6_af_pmc2 -o run -- python3 $R/tools/bc_step_probe.py > $R/gpurun_out/r6af_pmc2.log 2>&1 &&
cd $R && cp $(find /tmp/r6_af_pmc2 -name "*counter_collection.csv" | head -1) gpurun_out/r6af_pmc2.csv
rm -rf /tmp/r6_af_pmc /tmp/r6_af_pmc2

# one PMC pass (SQ counters only) over a short bench run; summary per kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --eval-episodes 0 > $GRAFT_REPO_ROOT/gpurun_out/pmc.log 2>&1 || { echo "pmc failed rc=$?"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc.log; exit 1; }
cd $GRAFT_REPO_ROOT && find gpurun_out/pmc -name "*.csv" | head
echo ALL OK

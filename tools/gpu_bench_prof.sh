# rocprof kernel trace of the headline bench (summary -> gpurun_out/prof_bench_summary.md) + SQ PMC pass
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bench -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_bench -name "*.db" | head -1) 25 > gpurun_out/prof_bench_summary.md
python tools/prof_timeline.py $(find gpurun_out/prof_bench -name "*.db" | head -1) rollout_chain_kernel 6 > gpurun_out/prof_bench_timeline.md || true
rm -rf gpurun_out/prof_bench
tail -1 gpurun_out/prof_bench.log
head -16 gpurun_out/prof_bench_summary.md
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --eval-episodes 0 > $GRAFT_REPO_ROOT/gpurun_out/pmc.log 2>&1 || { echo "pmc failed rc=$?"; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py $(find gpurun_out/pmc -name "*counter_collection.csv" | head -1) 8 > gpurun_out/pmc_bench_summary.md && head -6 gpurun_out/pmc_bench_summary.md

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/bc_step_probe.py 2>&1 | grep -v Warn | tail -2
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bc -o run -- python3 $GRAFT_REPO_ROOT/tools/bc_step_probe.py > $GRAFT_REPO_ROOT/gpurun_out/prof_bc.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_bc.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_bc -name "*.db" | head -1) 60 > gpurun_out/prof_bc_summary.md
rm -rf gpurun_out/prof_bc
cat gpurun_out/prof_bc_summary.md

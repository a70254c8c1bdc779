set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/cnn_bc_probe.py 2>&1 | grep -v Warn
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_cnn -o run -- python $GRAFT_REPO_ROOT/tools/cnn_bc_probe.py > $GRAFT_REPO_ROOT/gpurun_out/prof_cnn.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_cnn.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_cnn -name "*.db" | head -1) 40 > gpurun_out/prof_cnn_summary.md
rm -rf gpurun_out/prof_cnn
head -44 gpurun_out/prof_cnn_summary.md

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_ck -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_kprobe.py > $GRAFT_REPO_ROOT/gpurun_out/prof_ck.log 2>&1 || { echo "prof failed rc=$?"; tail $GRAFT_REPO_ROOT/gpurun_out/prof_ck.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_ck -name "*.db" | head -1) 25 > gpurun_out/prof_ck_summary.md
rm -rf gpurun_out/prof_ck
head -30 gpurun_out/prof_ck_summary.md

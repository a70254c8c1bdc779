set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_dagger -o run -- python $GRAFT_REPO_ROOT/tools/dagger_probe.py > $GRAFT_REPO_ROOT/gpurun_out/prof_dagger.log 2>&1 || { echo "prof failed rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_dagger.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $(find gpurun_out/prof_dagger -name "*.db" | head -1) 30 > gpurun_out/prof_dagger_summary.md
rm -rf gpurun_out/prof_dagger
grep round gpurun_out/prof_dagger.log; head -34 gpurun_out/prof_dagger_summary.md

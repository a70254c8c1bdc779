set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/dagger_probe.py > gpurun_out/dagger_probe.log 2>&1; echo rc=$?
grep -v "Saving the dataset\|Warn" gpurun_out/dagger_probe.log | head -80

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/dagger_probe.py > gpurun_out/dagger_probe.log 2>&1 || { echo "probe failed rc=$?"; tail -30 gpurun_out/dagger_probe.log; exit 1; }
grep -v Warn gpurun_out/dagger_probe.log | tail -60 | cut -c1-180

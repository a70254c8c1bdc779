set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PROBE_CPROFILE=1 timeout -k 10 300 python tools/pref_rm_probe.py > gpurun_out/pref_cold.log 2>&1 && grep -E "cold call|reward training" gpurun_out/pref_cold.log

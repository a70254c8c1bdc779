#!/bin/bash
# round 6 call S: BC-step kernel trace on the final BC build (grids / times per kernel), BC head phases
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6s_bcprof -o bc -- python3 $R/tools/bc_step_probe.py > $R/gpurun_out/r6s_bcprof.log 2>&1 || exit $?
cd $R && timeout -k 10 120 python -u tools/bc_head_probe.py > gpurun_out/r6s_head.log 2>&1 || exit $?

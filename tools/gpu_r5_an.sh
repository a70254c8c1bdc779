#!/bin/bash
# round 5, call AN: end-of-round kernel tables (rocprofv3 --kernel-trace --stats) of the headline bench, AIRL and DRLHP
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
prof() {  # name, command...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r5_an_$name -o run -- "$@" > gpurun_out/r5_an_$name.log 2>&1 || return 1
  timeout -k 10 120 python3 tools/prof_summary.py $(ls /tmp/r5_an_$name/*.db | head -1) > gpurun_out/r5_an_${name}_kernels.md
  local rc=$?
  rm -rf /tmp/r5_an_$name
  return $rc
}
prof gail python3 bench.py --steps 20 --warmup 3 &&
prof airl python3 benchmarking/bench_configs.py --configs airl_hopper --steps 6 --warmup 2 &&
prof drlhp python3 benchmarking/bench_configs.py --configs preference_walker2d --steps 2 --warmup 1

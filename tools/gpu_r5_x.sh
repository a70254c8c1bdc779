#!/bin/bash
# round 5, call X: ROCTX phase timelines (IMITATION_AMD_ROCTX=1, rocprofv3 --kernel-trace --marker-trace) of
# GAIL, AIRL, DRLHP and DAgger rounds, summarised on the box (the databases are too large to copy back)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp IMITATION_AMD_ROCTX=1
run() {  # name, round range, nth, command...
  local name=$1 rr=$2 nth=$3; shift 3
  timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace -d /tmp/r5_x_$name -o run -- "$@" > gpurun_out/r5_x_$name.log 2>&1 || return 1
  timeout -k 10 120 python3 tools/roctx_summary.py $(ls /tmp/r5_x_$name/*.db | head -1) --round-range "$rr" --nth $nth > gpurun_out/r5_x_$name.md 2>&1
  local rc=$?
  rm -rf /tmp/r5_x_$name
  return $rc
}
run gail ppo/update 12 python3 bench.py --steps 30 --warmup 3 &&
run airl ppo/update 4 python3 benchmarking/bench_configs.py --configs airl_hopper --steps 6 --warmup 2 &&
run drlhp pref/agent_train 1 python3 benchmarking/bench_configs.py --configs preference_walker2d --steps 2 --warmup 1 &&
run dagger dagger/collect 2 python3 benchmarking/bench_configs.py --configs dagger_pong --steps 3 --warmup 1

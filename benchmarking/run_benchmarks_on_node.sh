#!/bin/bash
# Run the benchmark commands on one 8-GPU MI355X node: one command per GPU at a time.
# Usage: benchmarking/run_benchmarks_on_node.sh [commands_file]   (default: run_all_benchmarks.sh)
set -u
CMDS=${1:-$(dirname "$0")/run_all_benchmarks.sh}
NGPU=${NGPU:-8}
grep '^python' "$CMDS" | awk -v n="$NGPU" '{print (NR-1)%n "\t" $0}' | \
  xargs -P "$NGPU" -d '\n' -I{} bash -c 'line="{}"; gpu="${line%%$'"'"'\t'"'"'*}"; cmd="${line#*$'"'"'\t'"'"'}"; HIP_VISIBLE_DEVICES=$gpu $cmd'

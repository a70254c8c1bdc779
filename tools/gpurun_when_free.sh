#!/bin/bash
# Start a gpurun call, retrying ONLY while the pool reports no free box / slot (exit 3: nothing ran,
# nothing charged). Any other exit (success, refusal, a failed or timed-out GPU step) ends it.
# usage: tools/gpurun_when_free.sh <gpurun timeout s> <command...>
T=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  if [ $rc -ne 3 ]; then exit $rc; fi
  echo "[gpurun_when_free] no free box (attempt $i), waiting 120 s" >&2
  sleep 120
done
exit 3

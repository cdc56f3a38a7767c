#!/bin/bash
# Submit one gpurun call, re-submitting only while the pool reports no free slot/box
# (nothing ran, nothing charged); any other outcome ends the loop.
# Usage: bash scripts/gpurun_wait.sh OUTFILE TIMEOUT -- command...
out=$1; to=$2; shift 3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { [ $rc -eq 2 ] && grep -q "busy\|no free box" "$out"; }; then sleep 60; continue; fi
  exit $rc
done

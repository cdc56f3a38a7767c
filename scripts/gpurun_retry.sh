#!/bin/bash
# Host-side helper: run ONE gpurun call, re-submitting it only when gpurun
# reports an infrastructure event (no slot free / box taken away: nothing ran,
# nothing charged).  A call that ran -- whatever its exit status -- is never
# repeated.  Usage: bash scripts/gpurun_retry.sh OUT.txt TIMEOUT -- CMD...
OUT=$1; TMO=$2; shift 3
for attempt in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$@" > "$OUT" 2>&1
  rc=$?
  if grep -q "status=transient\|slot(s) on this pod are busy\|backing off" "$OUT" && ! grep -q "status=ok\|status=fail" "$OUT"; then
    echo "attempt $attempt: infrastructure event, retrying in 120 s" >> "$OUT.retries"
    sleep 120
    continue
  fi
  exit $rc
done
exit 3

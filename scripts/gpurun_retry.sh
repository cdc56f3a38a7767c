#!/bin/bash
# Host-side helper: run ONE gpurun call, re-submitting it only when gpurun
# reports an infrastructure event (no slot free / box taken away: nothing ran,
# nothing charged).  A call that ran -- whatever its exit status -- is never
# repeated.  Usage: bash scripts/gpurun_retry.sh OUT.txt TIMEOUT -- CMD...
OUT=$1; TMO=$2; shift 3
for attempt in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$@" > "$OUT" 2>&1
  rc=$?
  if grep -q "status=transient\|slot(s) on this pod are busy\|backing off" "$OUT" && ! grep -q "status=ok\|status=fail" "$OUT"; then
    wait_s=$(grep -o "retry in [0-9]*s" "$OUT" | grep -o "[0-9]*" | tail -1)
    wait_s=${wait_s:-120}
    [ "$wait_s" -lt 120 ] && wait_s=120
    echo "attempt $attempt: infrastructure event, retrying in $wait_s s" >> "$OUT.retries"
    sleep $wait_s
    continue
  fi
  exit $rc
done
exit 3

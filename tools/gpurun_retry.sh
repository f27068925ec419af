#!/bin/bash
# gpurun with retries while the pool has no free box ("status=transient" or "has no free box": nothing
# ran, nothing charged).  Any other outcome -- success, a failing command, a
# refusal -- ends the loop.  Usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -qE "status=transient|has no free box" "$log"; then
    echo "[retry $i: transient, sleeping]" >> "$log.retries"
    sleep 150
    continue
  fi
  exit $rc
done
echo "[gpurun_retry: no box after 12 tries]" >> "$log"
exit 3

#!/bin/bash
# Submit ONE gpurun command, resubmitting only when the pool refused it before anything ran (no free
# box, back-off, box lost while being prepared: nothing charged, nothing executed).  A command that ran
# is never resubmitted, whatever its exit status.  usage: tools/gpu_try.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q -E "no free box|backing off|stopped responding while being prepared|taken away by the GPU service|slot\(s\) on this pod are busy" "$LOG" && ! grep -q "status=ok\|status=fail" "$LOG"; then
    sleep 150
    continue
  fi
  exit $rc
done
exit 3

#!/bin/bash
# Retry a gpurun call ONLY when nothing ran on a GPU: no box/slot free (exit 3) or an
# infrastructure-side transient (box lost while being prepared, back-off; "status=transient",
# nothing charged).  A command that ran -- whatever its exit code -- is never retried.
# Usage: tools/gpurun_retry.sh LOGFILE TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
    timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
    rc=$?
    echo "[retry] attempt $i rc=$rc" >> "$LOG"
    if [ "$rc" -ne 3 ] && ! grep -q "status=transient" "$LOG"; then exit "$rc"; fi
    sleep 60
done
exit 3

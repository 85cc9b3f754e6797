#!/bin/bash
# Retry a gpurun call ONLY when no box/slot was free (exit 3: nothing ran, nothing charged).
# Usage: tools/gpurun_retry.sh LOGFILE TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8 9 10; do
    timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
    rc=$?
    echo "[retry] attempt $i rc=$rc" >> "$LOG"
    [ "$rc" -ne 3 ] && exit "$rc"
    sleep 60
done
exit 3

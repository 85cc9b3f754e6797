#!/bin/bash
# Retry a gpurun call ONLY when nothing ran on a GPU: no box/slot free (exit 3) or an
# infrastructure-side transient (box lost while being prepared, back-off; "status=transient",
# nothing charged).  A command that ran -- whatever its exit code -- is never retried.
# Waits as long as gpurun's back-off message asks ("retry in Ns"), at least 60 s.
# Usage: tools/gpurun_retry.sh LOGFILE TIMEOUT 'command' [ATTEMPTS]
LOG=$1; TO=$2; CMD=$3; N=${4:-20}
for i in $(seq 1 "$N"); do
    timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
    rc=$?
    echo "[retry] attempt $i rc=$rc" >> "$LOG"
    if [ "$rc" -ne 3 ] && ! grep -q "status=transient" "$LOG"; then exit "$rc"; fi
    w=$(grep -o "retry in [0-9]*s" "$LOG" | tail -1 | grep -o "[0-9]*")
    w=${w:-60}; [ "$w" -lt 60 ] && w=60
    sleep $((w + 10))
done
exit 3

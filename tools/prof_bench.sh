#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv \
    -- python3 bench.py --steps "${STEPS:-10}" --warmup 2 --no-cpu-baseline "$@" \
    > "$OUT.json" 2> "$OUT.err"
echo "rocprof exit $?"
cat "$OUT.json"

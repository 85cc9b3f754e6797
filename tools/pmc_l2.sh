#!/bin/bash
# L2 hit / miss of the bench workload's kernels (one rocprofv3 --pmc pass of its own, no trace
# domains): TCC_HIT_sum, TCC_MISS_sum per dispatch.  Output under gpurun_out/prof_$ROUND/l2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
ROUND=${ROUND:-r02}
OUT=gpurun_out/prof_$ROUND
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/l2" -o run --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$OUT/l2_bench.json" \
    2> "$OUT/l2_bench.err" || { echo "L2 pass failed ($?)"; exit 1; }
echo "L2 pass ok"

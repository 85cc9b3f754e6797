#!/bin/bash
# Round profile of the bench workload (run on the GPU box):
#   1. rocprofv3 --kernel-trace --stats       -> per-kernel average durations
# every pass over the same bench window, STEPS timed sweeps after WARMUP (default the
# driver's 20 after 5), recorded in the summary: bench.py matches the per-sweep kernels'
# traffic on it (a kernel's average over its dispatches depends on the window's regime)
#   2. rocprofv3 --pmc FETCH_SIZE  (own pass) -> HBM read KB per dispatch
#   3. rocprofv3 --pmc WRITE_SIZE  (own pass) -> HBM write KB per dispatch
# No --pmc pass is combined with any trace domain.  Each step has its own time limit and
# a failure ends the script.  Summaries: python tools/profile_summary.py <round>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
ROUND=${ROUND:-r01}
OUT=gpurun_out/prof_$ROUND
mkdir -p "$OUT"
# the sources this profile measures (bench.py uses a profile only for the same tree)
python3 -c "from bayesbridge_amd._build import source_sha; print(source_sha())" > "$OUT/source_sha.txt"
# and the code identity of every kernel in the library it runs (bayesbridge_amd/_kernel_code.py)
python3 -m bayesbridge_amd._kernel_code > "$OUT/kernel_code.json" || exit 1
ARGS="--no-cpu-baseline $*"
WIN="--steps ${STEPS:-20} --warmup ${WARMUP:-5}"
set -o pipefail
# PASS=kt|fetch|write runs that one pass (one GPU step per call); unset: all three in turn
PASS=${PASS:-all}
if [ "$PASS" = all ] || [ "$PASS" = kt ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv \
    -- python3 bench.py $WIN $ARGS > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" \
    || { echo "kernel-trace pass failed ($?)"; exit 1; }
echo "kernel-trace pass ok"
fi
if [ "$PASS" = all ] || [ "$PASS" = fetch ]; then
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
    -- python3 bench.py $WIN $ARGS > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err" \
    || { echo "FETCH_SIZE pass failed ($?)"; exit 1; }
echo "FETCH_SIZE pass ok"
fi
if [ "$PASS" = all ] || [ "$PASS" = write ]; then
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
    -- python3 bench.py $WIN $ARGS > "$OUT/write_bench.json" 2> "$OUT/write_bench.err" \
    || { echo "WRITE_SIZE pass failed ($?)"; exit 1; }
echo "WRITE_SIZE pass ok"
fi

#!/bin/bash
# Round-4 session ab: k_pre with eight loads in flight per thread -- the whole GPU suite,
# C3 at the driver's settings three times, and a C3 kernel trace (k_pre's duration).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r04ab_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/r04ab_tests.log | tail -6
stop tests $rc
for r in 1 2 3; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted \
        > gpurun_out/r04ab_c3_$r.json 2>> gpurun_out/r04ab_bench.err
    stop c3 $?
done
python3 - <<'PY'
import json
for r in (1, 2, 3):
    d = json.loads(open(f"gpurun_out/r04ab_c3_{r}.json").read().strip().splitlines()[-1])
    print("c3", round(d["value"], 1), d.get("phases_ms"))
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_ab" \
    -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-fitted \
    > "$GRAFT_REPO_ROOT/gpurun_out/r04ab_prof.log" 2>&1
stop prof $?
echo "[session] done"

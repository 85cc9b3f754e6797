#!/bin/bash
# Round-4 session ac: k_cheb_init over 4-row workgroups for >= 1024 partials (the fused
# launch's 1568 at C3) -- near-identity tests, C3 three times, a C3 kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_nid_gpu.py tests/test_shard_nid_gpu.py \
    tests/test_steady_state_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r04ac_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/r04ac_tests.log | tail -4
stop tests $rc
for r in 1 2 3; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted \
        > gpurun_out/r04ac_c3_$r.json 2>> gpurun_out/r04ac_bench.err
    stop c3 $?
done
python3 - <<'PY'
import json
for r in (1, 2, 3):
    d = json.loads(open(f"gpurun_out/r04ac_c3_{r}.json").read().strip().splitlines()[-1])
    print("c3", round(d["value"], 1), d.get("phases_ms"))
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_ac" \
    -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-fitted \
    > "$GRAFT_REPO_ROOT/gpurun_out/r04ac_prof.log" 2>&1
stop prof $?
echo "[session] done"

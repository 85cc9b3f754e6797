#!/bin/bash
# Round-4 session w: the decision sums back to two launches; non-temporal partial stores;
# Chebyshev partial sums -- near-identity / parity / sparse / shard / steady-state GPU tests,
# C3 / C5 / C2 bench lines and a C3 kernel trace (the per-sweep small kernels).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_nid_gpu.py tests/test_shard_nid_gpu.py \
    tests/test_gpu_parity.py tests/test_sparse_gpu.py tests/test_steady_state_gpu.py -m gpu -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04w_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04w_tests.log
stop tests $rc
for r in 1 2; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted \
        > gpurun_out/r04w_c3_$r.json 2>> gpurun_out/r04w_bench.err
    stop c3 $?
done
timeout -k 10 300 python -u bench.py --workload c5 --steps 200 --warmup 20 --no-cpu-baseline \
    --no-fitted > gpurun_out/r04w_c5.json 2>> gpurun_out/r04w_bench.err
stop c5 $?
timeout -k 10 300 python -u bench.py --workload c2 --no-cpu-baseline --no-fitted \
    > gpurun_out/r04w_c2.json 2>> gpurun_out/r04w_bench.err
stop c2 $?
python3 - <<'PY'
import json
for w in ["c3_1", "c3_2", "c5", "c2"]:
    try:
        d = json.loads(open(f"gpurun_out/r04w_{w}.json").read().strip().splitlines()[-1])
    except Exception as ex:
        print(w, "no line", ex)
        continue
    print(w, round(d["value"], 1), round(d["ms_per_step"], 4), d.get("phases_ms"))
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_w" \
    -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-fitted \
    > "$GRAFT_REPO_ROOT/gpurun_out/r04w_prof.log" 2>&1
stop prof $?
echo "[session] done"

#!/bin/bash
# Round-4 session y: the host polls the synchronous decision's tag instead of waiting on an
# event (bb_set_tuning key 10) -- GPU tests of the paths that take the protocol (single
# engines, shard groups, the .C driver), then C3 at the driver's settings with the tag (10=1)
# and with the event (10=0), alternated, and C5 / C2 once.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_nid_gpu.py tests/test_shard_nid_gpu.py \
    tests/test_gpu_parity.py tests/test_sparse_gpu.py tests/test_driver_gpu.py \
    tests/test_steady_state_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r04y_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04y_tests.log
stop tests $rc
for r in 1 2 3; do
    for k in 1 0; do
        timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted \
            --tuning 10=$k > gpurun_out/r04y_c3_k${k}_$r.json 2>> gpurun_out/r04y_bench.err
        stop c3 $?
    done
done
timeout -k 10 300 python -u bench.py --workload c5 --steps 200 --warmup 20 --no-cpu-baseline \
    --no-fitted > gpurun_out/r04y_c5.json 2>> gpurun_out/r04y_bench.err
stop c5 $?
timeout -k 10 300 python -u bench.py --workload c2 --no-cpu-baseline --no-fitted \
    > gpurun_out/r04y_c2.json 2>> gpurun_out/r04y_bench.err
stop c2 $?
python3 - <<'PY'
import json
for k in (1, 0):
    vals = []
    for r in (1, 2, 3):
        d = json.loads(open(f"gpurun_out/r04y_c3_k{k}_{r}.json").read().strip().splitlines()[-1])
        vals.append(round(d["value"], 1))
    print("key10", k, vals)
for w in ("c5", "c2"):
    d = json.loads(open(f"gpurun_out/r04y_{w}.json").read().strip().splitlines()[-1])
    print(w, round(d["value"], 1), d.get("phases_ms"))
PY
echo "[session] done"

#!/bin/bash
# Round-4 session x: the wider Chebyshev partial sums (final form) and the timing stride --
# near-identity / shard GPU tests, then C3 at the driver's settings with the dominant kernel
# bracketed in every sweep (stride 1) and in every 4th (stride 4, the new default), alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_nid_gpu.py tests/test_shard_nid_gpu.py -m gpu -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04x_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04x_tests.log
stop tests $rc
for r in 1 2 3; do
    for s in 1 4; do
        timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted \
            --timing-stride $s > gpurun_out/r04x_c3_s${s}_$r.json 2>> gpurun_out/r04x_bench.err
        stop c3 $?
    done
done
python3 - <<'PY'
import json
for s in (1, 4):
    vals = []
    for r in (1, 2, 3):
        d = json.loads(open(f"gpurun_out/r04x_c3_s{s}_{r}.json").read().strip().splitlines()[-1])
        vals.append(round(d["value"], 1))
        ro = d["roofline"]
    print("stride", s, vals, ro.get("kernel"), round(ro.get("achieved") or 0, 1), ro.get("timing"))
PY
echo "[session] done"

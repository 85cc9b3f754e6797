#!/bin/bash
# Round-4 session e: the changed GPU tests, the pivot-latency microbenchmark, bench lines at
# the driver's settings (C3 with the fused lambda + X u launch on / off, C2, C5), and the C5
# round profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_nid_gpu.py tests/test_shard_nid_gpu.py \
    "tests/test_steady_state_gpu.py::test_fitted_regime_teacher_forced" \
    -m gpu -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r04e_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|fitted start|worst" gpurun_out/r04e_tests.log | tail -20
stop tests $rc
timeout -k 10 60 ./tools/chain_lat > gpurun_out/r04e_chain_lat.txt 2>&1
stop chain_lat $?
cat gpurun_out/r04e_chain_lat.txt
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted"
for r in 1 2; do
    timeout -k 10 300 $B > gpurun_out/r04e_c3_fused$r.json 2>> gpurun_out/r04e_bench.err
    stop c3_fused $?
    timeout -k 10 300 $B --tuning 7=0 > gpurun_out/r04e_c3_sep$r.json 2>> gpurun_out/r04e_bench.err
    stop c3_sep $?
done
timeout -k 10 300 $B --workload c2 > gpurun_out/r04e_c2.json 2>> gpurun_out/r04e_bench.err
stop c2 $?
timeout -k 10 300 $B --workload c5 > gpurun_out/r04e_c5.json 2>> gpurun_out/r04e_bench.err
stop c5 $?
python3 - <<'PY'
import json
for f in ["c3_fused1", "c3_sep1", "c3_fused2", "c3_sep2", "c2", "c5"]:
    d = json.loads(open(f"gpurun_out/r04e_{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["value"], 1), d["phases_ms"].get("lambda"), d["phases_ms"].get("nid"),
          d["roofline"].get("kernel"), d["roofline"].get("frac"))
PY
ROUND=r04c5 bash tools/profile_round.sh --workload c5 --no-fitted
stop prof_c5 $?
echo "[session] done"

#!/bin/bash
# Round-4 session f: near-identity tests (synchronous-decision mode added), bench lines at the
# driver's settings (C3: default / synchronous decision / separate lambda and X u, twice;
# C2, C5), and the C5 round profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_nid_gpu.py -m gpu -v -s -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/r04f_tests.log | tail -10
stop tests $rc
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted"
for r in 1 2; do
    timeout -k 10 300 $B > gpurun_out/r04f_c3_def$r.json 2>> gpurun_out/r04f_bench.err
    stop c3_def $?
    timeout -k 10 300 $B --tuning 8=1 > gpurun_out/r04f_c3_sync$r.json 2>> gpurun_out/r04f_bench.err
    stop c3_sync $?
    timeout -k 10 300 $B --tuning 7=0 > gpurun_out/r04f_c3_sep$r.json 2>> gpurun_out/r04f_bench.err
    stop c3_sep $?
done
for w in c2 c5; do
    timeout -k 10 300 $B --workload $w > gpurun_out/r04f_${w}_def.json 2>> gpurun_out/r04f_bench.err
    stop ${w}_def $?
    timeout -k 10 300 $B --workload $w --tuning 8=1 > gpurun_out/r04f_${w}_sync.json 2>> gpurun_out/r04f_bench.err
    stop ${w}_sync $?
done
python3 - <<'PY'
import json
for f in ["c3_def1", "c3_sync1", "c3_sep1", "c3_def2", "c3_sync2", "c3_sep2", "c2_def", "c2_sync",
          "c5_def", "c5_sync"]:
    try:
        d = json.loads(open(f"gpurun_out/r04f_{f}.json").read().strip().splitlines()[-1])
    except Exception as ex:
        print(f, "no line", ex)
        continue
    print(f, round(d["value"], 1), d["phases_ms"].get("lambda"), d["phases_ms"].get("nid"),
          d["roofline"].get("kernel"), d["roofline"].get("frac"))
PY
ROUND=r04c5 bash tools/profile_round.sh --workload c5 --no-fitted
stop prof_c5 $?
echo "[session] done"

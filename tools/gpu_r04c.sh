#!/bin/bash
# Round-4 session c: the changed GPU tests, VALU PMC passes, the round profiles of C3 and C5
# (kernel trace + FETCH/WRITE passes, no fitted-regime run so the profile is one regime),
# and the C3 bench line at the driver's settings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_steady_state_gpu.py tests/test_driver_gpu.py \
    tests/test_nid_gpu.py -m gpu -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r04c_tests.log 2>&1
stop tests $?
grep -E "passed|failed|FAILED|fitted start|state after|worst" gpurun_out/r04c_tests.log | tail -20
bash tools/pmc_valu.sh
stop pmc_valu $?
ROUND=r04 bash tools/profile_round.sh --no-fitted
stop prof_c3 $?
ROUND=r04c5 bash tools/profile_round.sh --workload c5 --no-fitted
stop prof_c5 $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04c_bench_c3d.json 2> gpurun_out/r04c_bench_c3d.err
stop bench $?
python3 -c "
import json; d=json.loads(open('gpurun_out/r04c_bench_c3d.json').read().strip().splitlines()[-1])
print(round(d['value'],1), d['roofline'].get('kernel'), d['roofline'].get('frac'), (d.get('fitted_regime') or {}).get('value'))"
echo "[session] done"

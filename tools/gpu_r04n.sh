#!/bin/bash
# Round-4 session n: lambda occupancy A/B after the uniform-constant change (key 4 = 4: the
# fused / speculative launches at 3 waves per SIMD; 5: at 4 waves, 128 VGPRs with spills),
# C3 and C2, plus the lambda / near-identity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_lambda_occ_gpu.py tests/test_nid_gpu.py \
    tests/test_gpu_parity.py -m gpu -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r04n_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/r04n_tests.log | tail -10
stop tests $rc
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted"
run() {
    local name=$1; shift
    timeout -k 10 300 $B "$@" > gpurun_out/r04n_$name.json 2>> gpurun_out/r04n_bench.err
    stop $name $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04n_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['value'],1), d['phases_ms'].get('lambda'))"
}
for r in 1 2; do
    run c3_o3_$r --tuning 4=4
    run c3_o4_$r --tuning 4=5
    run c2_o3_$r --workload c2 --tuning 4=4
    run c2_o4_$r --workload c2 --tuning 4=5
    run c5_$r --workload c5
done
echo "[session] done"

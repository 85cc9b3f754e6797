#!/bin/bash
# Round-4 session k: lambda variants -- the fused launch batched (key 7 = 3) against one chunk
# per workgroup (2) at C3 / C2, k_lambda_cb inlined (key 4 = 4) against out of line at 4 waves
# (2) at C5 -- after their bit-equality tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_steady_state_gpu.py tests/test_lambda_occ_gpu.py tests/test_nid_gpu.py tests/test_shard_nid_gpu.py tests/test_sparse_gpu.py \
    -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/r04k_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/r04k_tests.log | tail -10
stop tests $rc
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted"
run() {  # name, args
    local name=$1; shift
    timeout -k 10 300 $B "$@" > gpurun_out/r04k_$name.json 2>> gpurun_out/r04k_bench.err
    local rc=$?
    stop $name $rc
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04k_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['value'],1), d['phases_ms'].get('lambda'))"
}
for r in 1 2; do
    run c3_m2_$r --tuning 7=2
    run c3_m3_$r --tuning 7=3
    run c5_o2_$r --workload c5 --tuning 4=2
    run c5_o4_$r --workload c5 --tuning 4=4
    run c3_s1_$r --tuning 8=1
    run c3_s2_$r --tuning 8=2
    run c2_m2_$r --workload c2 --tuning 7=2
    run c2_m3_$r --workload c2 --tuning 7=3
done
echo "[session] done"

#!/bin/bash
# Round-4 session m: CSR row passes a wave per row with four accumulators: sparse GPU tests,
# then C5 bench lines at the driver's settings (three).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_sparse_gpu.py tests/test_nid_gpu.py \
    tests/test_shard_nid_gpu.py -m gpu -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r04m_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/r04m_tests.log | tail -10
stop tests $rc
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted"
for r in 1 2 3; do
    timeout -k 10 300 $B --workload c5 > gpurun_out/r04m_c5_$r.json 2>> gpurun_out/r04m_bench.err
    stop c5 $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04m_c5_$r.json').read().strip().splitlines()[-1])
print('c5', round(d['value'],1), d['phases_ms'])"
done
echo "[session] done"

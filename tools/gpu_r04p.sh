#!/bin/bash
# Round-4 session p: the small chain's one-barrier Cholesky with one rsqrt per pivot -- its GPU tests (small-p chains
# against the oracle, the published-ESS DB row) and C1 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "small or ortho or unknown or diabetes or golden or retstable" \
    -m gpu -v -p no:cacheprovider --timeout 600 \
    --timeout-method thread > gpurun_out/r04p_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ESS" gpurun_out/r04p_tests.log | tail -12
stop tests $rc
for r in 1 2; do
    timeout -k 10 300 python -u bench.py --workload c1 --steps 20000 --warmup 2000 --no-cpu-baseline \
        > gpurun_out/r04p_c1_$r.json 2>> gpurun_out/r04p_bench.err
    stop c1 $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04p_c1_$r.json').read().strip().splitlines()[-1])
print('c1', round(d['value'],1))"
done
echo "[session] done"

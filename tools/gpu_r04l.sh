#!/bin/bash
# Round-4 session l: CSR row passes one workgroup per row, S_alpha summed by the workgroup:
# the sparse / parity / steady-state / near-identity GPU tests, then bench lines (C5, C3, C2,
# C4) at the driver's settings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_sparse_gpu.py tests/test_gpu_parity.py \
    tests/test_steady_state_gpu.py tests/test_nid_gpu.py tests/test_shard_nid_gpu.py \
    tests/test_lambda_occ_gpu.py tests/test_logit_gpu.py \
    -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/r04l_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/r04l_tests.log | tail -10
stop tests $rc
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted"
for w in c5 c3 c2 c4 c5 c3; do
    timeout -k 10 300 $B --workload $w > gpurun_out/r04l_$w.json 2>> gpurun_out/r04l_bench.err
    stop $w $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04l_$w.json').read().strip().splitlines()[-1])
print('$w', round(d['value'],1), d['phases_ms'])"
done
echo "[session] done"

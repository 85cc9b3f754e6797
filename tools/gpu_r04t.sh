#!/bin/bash
# Round-4 session t: the batching lambda launch at C3's p by default -- lambda / parity /
# steady-state GPU tests, then C3 bench lines (with the fitted-regime run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_lambda_occ_gpu.py tests/test_gpu_parity.py \
    tests/test_steady_state_gpu.py tests/test_nid_gpu.py -m gpu -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/r04t_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r04t_tests.log
stop tests $rc
for r in 1 2; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/r04t_c3_$r.json 2>> gpurun_out/r04t_bench.err
    stop c3 $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04t_c3_$r.json').read().strip().splitlines()[-1])
f=d['fitted_regime']; print('c3', round(d['value'],1), 'fitted', round(f['value'],1), f['phases_ms'].get('lambda'))"
done
echo "[session] done"

#!/bin/bash
# Round-4 session s: the separate lambda launch at C3's p (the fitted regime): speculative
# k_lambda_spec<8> (key 4 = 4, default) against the inlined continuous-batching launch
# (key 4 = 12), read from bench's fitted-regime phase split; plus the lambda variant tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_lambda_occ_gpu.py -m gpu -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/r04s_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r04s_tests.log
stop tests $rc
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for r in 1 2; do
    for v in 4 12; do
        timeout -k 10 300 $B --tuning 4=$v > gpurun_out/r04s_c3_o$v$r.json 2>> gpurun_out/r04s_bench.err
        stop c3_o$v $?
        python3 -c "
import json; d=json.loads(open('gpurun_out/r04s_c3_o$v$r.json').read().strip().splitlines()[-1])
f=d['fitted_regime']; print('c3 key4=$v', round(d['value'],1), 'fitted', round(f['value'],1), f['phases_ms'].get('lambda'))"
    done
done
echo "[session] done"

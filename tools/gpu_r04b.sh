#!/bin/bash
# Round-4 session: near-identity tests first, the GPU suite, then bench lines (C3 at the
# driver's settings and the defaults, C5, C2).  Each GPU step is time-limited; a fault /
# abort / timeout ends the script (test failures do not).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_nid_gpu.py -m gpu -v -s -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/r04b_nid.log 2>&1
stop nid $?
grep -E "passed|failed|FAILED|Error|iterates|eps=" gpurun_out/r04b_nid.log | tail -40
if [ "${TESTS:-1}" = "1" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
        --timeout-method thread > gpurun_out/r04b_pytest_gpu.log 2>&1
    stop pytest $?
    grep -E "passed|failed|FAILED|ERROR" gpurun_out/r04b_pytest_gpu.log | tail -12
fi
for cfg in "c3d:--steps 20 --warmup 5" "c3:" "c5:--workload c5" "c2:--workload c2"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 600 python -u bench.py $args > gpurun_out/r04b_bench_$name.json 2> gpurun_out/r04b_bench_$name.err
    stop "bench $name" $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04b_bench_$name.json').read().strip().splitlines()[-1])
f=d.get('fitted_regime') or {}
print('$name', round(d['value'],1), 'ms', round(d['ms_per_step'],3), d['roofline'].get('kernel'), d['roofline'].get('frac'), 'nid', d.get('near_identity'), 'fitted', round(f.get('value',0),1), f.get('chebyshev_sweeps'))
print('   phases', d.get('phases_ms'))"
done
echo "[session] done"

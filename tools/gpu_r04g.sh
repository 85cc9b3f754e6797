#!/bin/bash
# Round-4 session g: the whole GPU suite (the sampler's outer test now takes A from the inner
# attempt's B / B0), bench lines at the driver's settings (C3, C5, C2), VALU PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r04g_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/r04g_tests.log | tail -15
stop tests $rc
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted"
for w in c3 c5 c2 c3; do
    timeout -k 10 300 $B --workload $w > gpurun_out/r04g_$w.json 2>> gpurun_out/r04g_bench.err
    stop $w $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04g_$w.json').read().strip().splitlines()[-1])
print('$w', round(d['value'],1), d['phases_ms'].get('lambda'), d['roofline'].get('kernel'), d['roofline'].get('frac'))"
done
bash tools/pmc_valu.sh
stop pmc_valu $?
echo "[session] done"

#!/bin/bash
# Round-4 session r: the whole GPU suite and smoke() on the current tree, then C3 (twice) and
# C5 bench lines at the driver's settings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r04r_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/r04r_tests.log | tail -15
stop tests $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/r04r_smoke.log 2>&1
stop smoke $?
tail -2 gpurun_out/r04r_smoke.log
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted"
for w in c3 c5 c3; do
    timeout -k 10 300 $B --workload $w > gpurun_out/r04r_$w.json 2>> gpurun_out/r04r_bench.err
    stop $w $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04r_$w.json').read().strip().splitlines()[-1])
print('$w', round(d['value'],1), d['phases_ms'])"
done
echo "[session] done"

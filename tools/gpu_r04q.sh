#!/bin/bash
# Round-4 session q: the small chain's factor variants A/B at C1 (key 9 = 1: one barrier per
# pivot; 0: the reference's order, two), three alternations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "small or ortho or unknown or diabetes" \
    -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r04q_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r04q_tests.log
stop tests $rc
for r in 1 2 3; do
    for v in 1 0; do
        timeout -k 10 300 python -u bench.py --workload c1 --steps 20000 --warmup 2000 --no-cpu-baseline \
            --tuning 9=$v > gpurun_out/r04q_c1_k$v$r.json 2>> gpurun_out/r04q_bench.err
        stop c1 $?
        python3 -c "
import json; d=json.loads(open('gpurun_out/r04q_c1_k$v$r.json').read().strip().splitlines()[-1])
print('c1 key9=$v', round(d['value'],1))"
    done
done
echo "[session] done"

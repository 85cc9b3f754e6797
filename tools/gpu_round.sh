#!/bin/bash
# Round-end evidence session (run on the GPU box): the full GPU test suite and smoke, then one
# bench line per BASELINE config into gpurun_out/bench_cK.json.  Each GPU step is
# time-limited; a fault / abort / timeout ends the script (test failures do not).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[round] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
if [ "${TESTS:-1}" = "1" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
        --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
    stop pytest $?
    grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -8
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    stop smoke $?
    tail -2 gpurun_out/smoke.log
fi
for wl in ${WORKLOADS:-c3 c2 c4 c5 c1}; do
    case $wl in
        c1) args="--workload c1 --steps 20000 --warmup 2000" ;;
        c5) args="--workload c5 --steps 200 --warmup 20" ;;
        *) args="--workload $wl --steps 1000 --warmup 100" ;;
    esac
    timeout -k 10 600 python -u bench.py $args > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err
    stop "bench $wl" $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$wl.json').read().strip().splitlines()[-1]); print('$wl', round(d['value'],1), d['roofline'].get('kernel'), d['roofline'].get('frac'))"
done
echo "[round] done"

#!/bin/bash
# One GPU session (round 3): the GPU tests (TESTS, default the whole -m gpu suite), then the
# bench lines listed in BENCHES (";"-separated argument lists for bench.py), each step under
# its own time limit.  A fault, abort, segfault or timeout ends the script; test failures
# (status 1) and expected refusals do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
ok_or_stop() {  # $1 = exit status, $2 = step name
    local rc=$1
    echo "[session] $2 exit $rc"
    if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then
        echo "[session] stopping after $2 (status $rc)"
        exit "$rc"
    fi
}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
    timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider \
        --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
    ok_or_stop $? pytest
    tail -40 gpurun_out/pytest_gpu.log | grep -v PASSED
    grep -E "steady state|worst over" gpurun_out/pytest_gpu.log
fi
i=0
IFS=';' read -ra BL <<< "${BENCHES:-}"
for b in "${BL[@]}"; do
    i=$((i + 1))
    timeout -k 10 600 python -u bench.py $b > gpurun_out/bench_$i.json 2> gpurun_out/bench_$i.err
    ok_or_stop $? "bench $i ($b)"
    cat gpurun_out/bench_$i.json
    tail -3 gpurun_out/bench_$i.err
done
echo "[session] done"

#!/bin/bash
# One GPU session: the GPU tests (TESTS, default the whole -m gpu suite; PYTEST_ARGS extra
# arguments, e.g. "-k shard"), then the bench lines listed in BENCHES (";"-separated argument
# lists for bench.py; leading VAR=VALUE words are exported for that bench only, e.g.
# "BB_FORCE_RCCL=1 --cols 6250 --no-fitted"), then the commands in EXTRA (";"-separated, run
# from the repo root).  Each step runs under its own time limit.  A fault, abort, segfault or
# timeout ends the script; test failures (status 1) and expected refusals do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
TAG=${TAG:-s}
ok_or_stop() {  # $1 = exit status, $2 = step name
    local rc=$1
    echo "[session] $2 exit $rc"
    if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then
        echo "[session] stopping after $2 (status $rc)"
        exit "$rc"
    fi
}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
    timeout -k 10 "${TEST_LIMIT:-900}" python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider \
        --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${TAG}_pytest.log 2>&1
    ok_or_stop $? pytest
    tail -40 gpurun_out/${TAG}_pytest.log | grep -v PASSED
    grep -E "steady state|worst over|\[C3 x8|forced shard" gpurun_out/${TAG}_pytest.log
fi
i=0
IFS=';' read -ra BL <<< "${BENCHES:-}"
for b in "${BL[@]}"; do
    i=$((i + 1))
    envs=()
    args=()
    for w in $b; do
        if [ ${#args[@]} -eq 0 ] && [[ "$w" =~ ^[A-Z_][A-Z0-9_]*=.*$ ]]; then envs+=("$w"); else args+=("$w"); fi
    done
    (
        for kv in "${envs[@]}"; do export "$kv"; done
        timeout -k 10 600 python -u bench.py "${args[@]}" > gpurun_out/${TAG}_bench_$i.json \
            2> gpurun_out/${TAG}_bench_$i.err
    )
    ok_or_stop $? "bench $i ($b)"
    cat gpurun_out/${TAG}_bench_$i.json
    tail -3 gpurun_out/${TAG}_bench_$i.err
done
IFS=';' read -ra XL <<< "${EXTRA:-}"
for x in "${XL[@]}"; do
    timeout -k 10 600 bash -c "$x"
    ok_or_stop $? "extra ($x)"
done
echo "[session] done"

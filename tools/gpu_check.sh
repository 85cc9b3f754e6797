#!/bin/bash
# One GPU session: parity tests, smoke, a short bench and a rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a fault, abort, segfault or timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-20}
WARM=${WARM:-3}

ok_or_stop() {  # $1 = exit status, $2 = step name; 0/1 (test failures) continue
    local rc=$1
    echo "[gpu_check] $2 exit $rc"
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
        echo "[gpu_check] stopping after $2 (status $rc)"
        exit "$rc"
    fi
}

timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 \
    > gpurun_out/pytest_gpu.log 2>&1
ok_or_stop $? pytest
tail -30 gpurun_out/pytest_gpu.log

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
ok_or_stop $? smoke
tail -3 gpurun_out/smoke.log

timeout -k 10 600 python bench.py --steps "$STEPS" --warmup "$WARM" \
    > gpurun_out/bench.json 2> gpurun_out/bench.err
ok_or_stop $? bench
cat gpurun_out/bench.json
tail -5 gpurun_out/bench.err

if [ "${PROFILE:-1}" = "1" ]; then
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run \
        --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline \
        > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
    ok_or_stop $? rocprof
    find gpurun_out/prof -name "*stats*" | head
fi
echo "[gpu_check] done"

#!/bin/bash
# Round-3 study session: the steady-state parity tests, the published-protocol ESS table,
# the small-chain phase split at C1, and a long kernel-traced C3 run (per-dispatch lambda /
# Cholesky durations as the chain moves from the beta ~ 0 transient to the fitted regime).
# Each GPU step under its own limit; a fault / abort / timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[study] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
if [ "${TESTS:-1}" = "1" ]; then
    timeout -k 10 600 python -u -m pytest tests/test_steady_state_gpu.py tests/test_logit_gpu.py \
        -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
        > gpurun_out/study_tests.log 2>&1
    stop tests $?
    grep -E "state after|worst over|passed|failed|FAIL" gpurun_out/study_tests.log
fi
if [ "${PHASES:-1}" = "1" ]; then
    for pp in "100 20" "442 10" "442 32"; do
        timeout -k 10 60 ./tools/small_phase_bench $pp 0 4000 >> gpurun_out/small_phases.txt 2>&1
        stop "small_phase_bench $pp" $?
    done
    cat gpurun_out/small_phases.txt
fi
if [ "${TRACE:-1}" = "1" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_c3 -o run --output-format csv \
        -- python3 bench.py --steps ${TRACE_STEPS:-2500} --warmup 5 --no-cpu-baseline \
        > gpurun_out/trace_c3.json 2> gpurun_out/trace_c3.err
    stop trace $?
    python3 tools/dispatch_series.py gpurun_out/trace_c3 k_lambda 30
    python3 tools/dispatch_series.py gpurun_out/trace_c3 k_chol_persistent 30
    python3 tools/dispatch_series.py gpurun_out/trace_c3 k_oz_gemm16u 30
fi
if [ "${ESS:-1}" = "1" ]; then
    timeout -k 10 900 python3 -u tools/published_ess.py > gpurun_out/published_ess.json \
        2> gpurun_out/published_ess.err
    stop published_ess $?
    grep -v "sim " gpurun_out/published_ess.err | tail -12
fi
echo "[study] done"

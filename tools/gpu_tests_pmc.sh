#!/bin/bash
# One GPU session: the GPU test suite (new tests first), then the MFMA-busy PMC passes.
# Each GPU step is time-limited; a fault / abort / timeout ends the script (test failures
# do not).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
if [ -n "${FIRST:-}" ]; then
    timeout -k 10 600 python -u -m pytest $FIRST -m gpu -v -p no:cacheprovider --timeout 300 \
        --timeout-method thread > gpurun_out/pytest_first.log 2>&1
    stop first $?
    grep -E "passed|failed|FAILED|ERROR|fitted|state after" gpurun_out/pytest_first.log | tail -20
fi
if [ "${TESTS:-1}" = "1" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
        --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
    stop pytest $?
    grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -12
fi
if [ "${PMC:-1}" = "1" ]; then
    bash tools/pmc_mfma.sh
    stop pmc $?
fi
echo "[session] done"

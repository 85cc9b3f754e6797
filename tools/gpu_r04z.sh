#!/bin/bash
# Round-4 session z: bench.py end to end under pytest (tests/test_bench_gpu.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bench_gpu.py -m gpu -v -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/r04z_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r04z_tests.log
echo "[session] tests exit $rc"

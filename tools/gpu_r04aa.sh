#!/bin/bash
# Round-4 session aa: the near-identity tests incl. the narrow dense partial-sum cases.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nid_gpu.py -m gpu -v -s -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/r04aa_tests.log 2>&1
rc=$?
grep -E "iterates|passed|failed|FAILED" gpurun_out/r04aa_tests.log | tail -20
echo "[session] tests exit $rc"

#!/bin/bash
# the whole GPU test suite in one process (time-limited), log under gpurun_out/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_suite.log 2>&1
rc=$?; tail -15 gpurun_out/full_suite.log; exit $rc

#!/bin/bash
# Round-4 final session 1: the whole GPU suite and smoke() on the final tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r04F_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/r04F_tests.log | tail -15
stop tests $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/r04F_smoke.log 2>&1
stop smoke $?
tail -3 gpurun_out/r04F_smoke.log
echo "[session] done"

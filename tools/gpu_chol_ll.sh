#!/bin/bash
# GPU session: the Cholesky tagged-word hand-offs (key 21) -- parity tests, the factor A/B at
# m = 1024 / 2048 / 4096, then C4 A/B (300 sweeps after 30)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$SKIPT" ]; then
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_bsolve_ll_gpu.py tests/test_logit_gpu.py "tests/test_gpu_parity.py::test_chol_chain_versions_match_numpy" > gpurun_out/cll_test.log 2>&1
rc=$?; tail -5 gpurun_out/cll_test.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -u tools/chol_ll_ab.py > gpurun_out/cll_ab.txt 2>&1 || exit 1
cat gpurun_out/cll_ab.txt
MODES="21=1 21=0 21=1 21=0" SKIPT=1 bash tools/gpu_ll.sh

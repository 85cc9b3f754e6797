#!/bin/bash
# Round-4 session d: the sharded near-identity solve (on-device shard groups) and the group /
# near-identity / driver tests, then session c's VALU PMC passes, round profiles and bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_shard_nid_gpu.py tests/test_nid_gpu.py \
    "tests/test_gpu_parity.py::test_shard_group_matches_single_engine" \
    "tests/test_gpu_parity.py::test_shard_group_cu_filling_system" \
    "tests/test_sparse_gpu.py::test_sparse_shard_group_matches_single_engine" \
    tests/test_driver_gpu.py tests/test_steady_state_gpu.py \
    -m gpu -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r04d_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|iterates|fitted start|worst" gpurun_out/r04d_tests.log | tail -40
stop tests $rc
bash tools/gpu_r04c_tail.sh

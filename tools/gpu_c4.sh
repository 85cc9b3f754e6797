# GPU session: chain v4 parity (every size) then the v1 / v4 factor A/B with v4's step stamps
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=tests/test_gpu_parity.py::test_chol_chain_versions_match_numpy
timeout -k 10 60 ./tools/c4_micro > gpurun_out/c4_micro.log 2>&1; cat gpurun_out/c4_micro.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "$T[40-4]" "$T[64-4]" "$T[128-4]" "$T[200-4]" "$T[1000-4]" "$T[2048-4]" "$T[5000-4]" \
  > gpurun_out/c4_test.log 2>&1
rc=$?
tail -4 gpurun_out/c4_test.log
if [ $rc -ne 0 ]; then exit $rc; fi
CHOL_VERSIONS=${CHOL_VERSIONS:-1,4} timeout -k 10 300 python -u tools/bench_chol_ab.py > gpurun_out/c4_ab.log 2>&1
rc=$?
tail -40 gpurun_out/c4_ab.log
exit $rc

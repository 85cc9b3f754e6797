#!/bin/bash
# A/B session (run on the GPU box): Cholesky chain v1 vs v4 (parity tests + factor times +
# group stamps), Ozaki K-rotation (Gram tests, lead A/B times, L2 misses in an own PMC pass),
# and the host-enqueue probe.  Each GPU step is time-limited; a fault / timeout ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
stop() { echo "[ab] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
if [ "${CHOL:-1}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "chol" -v -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_chol.log 2>&1
  stop pytest_chol $?
  grep -E "passed|failed" gpurun_out/ab/pytest_chol.log | tail -2
  CHOL_VERSIONS=${CHOL_VERSIONS:-1,4} timeout -k 10 300 python -u tools/bench_chol_ab.py > gpurun_out/ab/chol_ab.txt 2>&1
  stop chol_ab $?
  cat gpurun_out/ab/chol_ab.txt
fi
if [ "${OZ:-1}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "ozaki or gram" -v -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_oz.log 2>&1
  stop pytest_oz $?
  grep -E "passed|failed" gpurun_out/ab/pytest_oz.log | tail -2
  timeout -k 10 180 python -u tools/oz_lead_probe.py 10 > gpurun_out/ab/oz_lead_times.txt 2>&1
  stop oz_lead $?
  cat gpurun_out/ab/oz_lead_times.txt
  timeout -s KILL 180 rocprofv3 --pmc TCC_MISS_sum TCC_HIT_sum -d gpurun_out/ab/oz_l2 -o run --output-format csv \
      -- python3 tools/oz_lead_probe.py 3 > gpurun_out/ab/oz_lead_pmc.txt 2>&1
  stop oz_pmc $?
fi
if [ "${ENQ:-1}" = "1" ]; then
  timeout -k 10 400 python -u tools/enqueue_probe.py > gpurun_out/enqueue_probe.json 2> gpurun_out/enqueue_probe.err
  stop enqueue $?
  cat gpurun_out/enqueue_probe.json
fi
echo "[ab] done"

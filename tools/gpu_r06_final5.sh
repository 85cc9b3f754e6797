#!/bin/bash
# after the 16-lane fallback fix of the fused lambda launch: its parity tests, then the C2 and
# per-rank proxy bench lines (each step time-limited; a failure ends the script)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_nid_gpu.py tests/test_nid_fold_gpu.py tests/test_shard_nid_gpu.py tests/test_shard8_gpu.py \
  tests/test_steady_state_gpu.py tests/test_lambda_occ_gpu.py > gpurun_out/fin5_test.log 2>&1
rc=$?; tail -3 gpurun_out/fin5_test.log; [ $rc -ne 0 ] && exit $rc
run() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python -u bench.py "$@" > gpurun_out/fin_$name.json 2> gpurun_out/fin_$name.err || exit 1
  echo "[fin] $name ok"
}
BB_FORCE_RCCL=1 run c3_rank_proxy 200 --cols 6250 --steps 20 --warmup 5 --no-cpu-baseline --no-fitted --tuning 16=2
BB_FORCE_RCCL=1 run c3_rank_proxy_own_chain 200 --cols 6250 --steps 20 --warmup 5 --no-cpu-baseline --no-fitted
run c2 400 --workload c2
run c3_driver 300 --steps 20 --warmup 5

#!/bin/bash
# Round-6 closing bench lines on the final tree (each step time-limited; a failure ends the
# script): C3 at the driver's settings and the defaults, the per-rank proxy, C4, C2 and C5
# (200 after 20) -- committed as profiles/r06_bench_*.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python -u bench.py "$@" > gpurun_out/fin_$name.json 2> gpurun_out/fin_$name.err || exit 1
  echo "[fin] $name ok"
}
run c3_driver 300 --steps 20 --warmup 5
run c3_default 600
BB_FORCE_RCCL=1 run c3_rank_proxy 200 --cols 6250 --steps 20 --warmup 5 --no-cpu-baseline --no-fitted --tuning 16=2
run c4 400 --workload c4
run c2 400 --workload c2
run c5_200 400 --workload c5 --steps 200 --warmup 20

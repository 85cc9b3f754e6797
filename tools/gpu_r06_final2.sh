#!/bin/bash
# Round-6 closing evidence after the folded bound sums (run on the GPU box; every step
# time-limited, a failure ends the script): the C3 profile passes (kernel trace, FETCH_SIZE,
# WRITE_SIZE, VALU counters) as round r06z, then the C3 bench lines -- the driver's settings
# (20 after 5) and the defaults (1000 after 100, with the fitted regime, the reference
# protocol and the CPU baselines) -- and the per-rank proxy.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$SKIPPROF" ]; then
PART=c3 ROUND=r06z bash tools/gpu_r06_final_prof.sh || exit 1
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/fin_c3_driver.json 2> gpurun_out/fin_c3_driver.err || exit 1
echo "[fin] driver line ok"
timeout -k 10 600 python -u bench.py > gpurun_out/fin_c3_default.json 2> gpurun_out/fin_c3_default.err || exit 1
echo "[fin] default line ok"
BB_FORCE_RCCL=1 timeout -k 10 200 python -u bench.py --cols 6250 --steps 20 --warmup 5 --no-cpu-baseline --no-fitted --tuning 16=2 > gpurun_out/fin_proxy.json 2> gpurun_out/fin_proxy.err || exit 1
echo "[fin] proxy line ok"

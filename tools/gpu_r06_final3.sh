#!/bin/bash
# Round-6 closing bench lines (run on the GPU box; every step time-limited, a failure ends the
# script): unless SKIPPROF, the C3 default-window profile passes (1000 after 100: kernel trace,
# FETCH_SIZE, WRITE_SIZE, round r06ze) that the default line's dominant kernel (k_eapply) is
# matched against; then the C3 lines at the driver's settings and the defaults, and the
# per-rank proxy.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$SKIPPROF" ]; then
for p in kt fetch write; do
    ROUND=r06ze STEPS=1000 WARMUP=100 PASS=$p bash tools/profile_round.sh --no-fitted || exit 1
done
fi
if [ -z "$SKIPLINES" ]; then
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/fin_c3_driver.json 2> gpurun_out/fin_c3_driver.err || exit 1
echo "[fin] driver line ok"
timeout -k 10 600 python -u bench.py > gpurun_out/fin_c3_default.json 2> gpurun_out/fin_c3_default.err || exit 1
echo "[fin] default line ok"
BB_FORCE_RCCL=1 timeout -k 10 200 python -u bench.py --cols 6250 --steps 20 --warmup 5 --no-cpu-baseline --no-fitted --tuning 16=2 > gpurun_out/fin_proxy.json 2> gpurun_out/fin_proxy.err || exit 1
echo "[fin] proxy line ok"
fi

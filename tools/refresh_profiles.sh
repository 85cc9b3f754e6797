#!/bin/bash
# Refresh one round's bench lines and rocprof summaries for the given workloads (run on the
# GPU box): bench.py line -> gpurun_out/bench_<wl>.json, then tools/profile_round.sh with
# ROUND=<round><suffix> (no suffix for c3, the headline).  Each GPU step is time-limited and
# a failure ends the script.  Then, here: python tools/profile_summary.py <round>[cK].
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
R=${ROUND:-r03}
for wl in ${WORKLOADS:-c3}; do
    case $wl in
        c1) args="--workload c1 --steps 20000 --warmup 2000" ;;
        c5) args="--workload c5 --steps 200 --warmup 20" ;;
        *) args="--workload $wl --steps 1000 --warmup 100" ;;
    esac
    timeout -k 10 600 python -u bench.py $args > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err \
        || { echo "bench $wl failed ($?)"; exit 1; }
    suf=$wl; [ "$wl" = c3 ] && suf=""
    ROUND=$R$suf timeout -k 10 900 bash tools/profile_round.sh --workload $wl \
        || { echo "profile $wl failed ($?)"; exit 1; }
    echo "[refresh] $wl done"
done

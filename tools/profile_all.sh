#!/bin/bash
# Round profile set (run on the GPU box): kernel-trace + FETCH_SIZE + WRITE_SIZE passes of the
# bench command for C3, C2, C4, C5 (tools/profile_round.sh, one pass per rocprofv3 run), the
# Ozaki pair-traffic probe (TCC_MISS/TCC_HIT in a pass of its own) and the host-enqueue probe.
# ROUND_PREFIX names the summaries (default r03).  Each step is time-limited; a failing step
# ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
P=${ROUND_PREFIX:-r03}
set -o pipefail
for wl in ${WORKLOADS:-c3 c2 c4 c5}; do
    r=$P; [ "$wl" != c3 ] && r=${P}${wl}
    ROUND=$r bash tools/profile_round.sh --workload $wl || { echo "profile $wl failed"; exit 1; }
    python3 tools/profile_summary.py $r > gpurun_out/summary_$r.txt 2>&1 || exit 1
    head -14 gpurun_out/summary_$r.txt
done
if [ "${OZPROBE:-1}" = "1" ]; then
    mkdir -p gpurun_out/ozprobe
    timeout -k 10 120 rocprofv3 --pmc TCC_MISS_sum TCC_HIT_sum -d gpurun_out/ozprobe/l2 -o run \
        --output-format csv -- python3 tools/oz_pairs_probe.py > gpurun_out/ozprobe/out.txt 2>&1 \
        || { echo "oz probe failed"; exit 1; }
    cat gpurun_out/ozprobe/out.txt | grep -v amdgpu.ids
fi
if [ "${ENQ:-1}" = "1" ]; then
    timeout -k 10 300 python3 tools/enqueue_probe.py > gpurun_out/enqueue_probe.json 2> gpurun_out/enqueue_probe.err \
        || { echo "enqueue probe failed"; exit 1; }
    cat gpurun_out/enqueue_probe.json
fi
echo "[profile_all] done"

#!/bin/bash
# Round-6 profile of the headline window (C3, the driver's 20 sweeps after 5): kernel trace,
# FETCH_SIZE, WRITE_SIZE (tools/profile_round.sh, one pass each) and the 14 VALU counters of
# the lambda launch (tools/pmc_valu.sh); every pass time-limited, a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=${ROUND:-r06x}
for p in kt fetch write; do
    ROUND=$R STEPS=20 WARMUP=5 PASS=$p bash tools/profile_round.sh --no-fitted || exit 1
done
ROUND=$R CONFIGS=c3 bash tools/pmc_valu.sh || exit 1
echo "[prof] done"

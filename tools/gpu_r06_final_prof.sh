#!/bin/bash
# Round-6 final profiles (run on the GPU box; each pass time-limited, a failure ends the script):
#   C3 headline window (20 after 5): kernel trace, FETCH_SIZE, WRITE_SIZE, the 14 VALU counters
#   C4 (1000 after 100): kernel trace, FETCH_SIZE, WRITE_SIZE; MFMA busy of the Cholesky
#   C5 (200 after 20): kernel trace, FETCH_SIZE, WRITE_SIZE, the 14 VALU counters
# Summaries here: tools/profile_summary.py r06y / r06yc4 / r06yc5, pmc_valu_summary.py r06y,
# pmc_mfma_summary.py r06y.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=${ROUND:-r06y}
if [ "${PART:-all}" = all ] || [ "$PART" = c3 ]; then
for p in kt fetch write; do
    ROUND=$R STEPS=20 WARMUP=5 PASS=$p bash tools/profile_round.sh --no-fitted || exit 1
done
ROUND=$R CONFIGS=c3 bash tools/pmc_valu.sh || exit 1
fi
if [ "${PART:-all}" = all ] || [ "$PART" = c4 ]; then
for p in kt fetch write; do
    ROUND=${R}c4 STEPS=1000 WARMUP=100 PASS=$p bash tools/profile_round.sh --workload c4 || exit 1
done
ROUND=$R CONFIGS=c4 bash tools/pmc_mfma.sh || exit 1
fi
if [ "${PART:-all}" = all ] || [ "$PART" = c5 ]; then
for p in kt fetch write; do
    ROUND=${R}c5 STEPS=200 WARMUP=20 PASS=$p bash tools/profile_round.sh --workload c5 --no-fitted || exit 1
done
ROUND=$R CONFIGS=c5 bash tools/pmc_valu.sh || exit 1
fi
echo "[prof] done"

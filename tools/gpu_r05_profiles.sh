#!/bin/bash
# Round-5 profiles of the final tree (run on the GPU box), PART selects a subset so each
# gpurun call stays within its limit:
#   PART=1  C3 at the driver's window (20 after 5, --no-fitted): kernel trace + FETCH/WRITE;
#           C3 at the bench defaults (1000 after 100, --no-fitted); C3 fitted (2 after 1, with
#           the fitted-regime run: the Gram, CRT and factor kernels)
#   PART=2  C5 (20 after 5), C4 and C2 (bench defaults, C2 --no-fitted) kernel traces + PMC
#   PART=3  VALU classes of the lambda launch (tools/pmc_valu.sh) and MFMA busy (pmc_mfma.sh)
# Summaries afterwards on the CPU: tools/profile_summary.py, pmc_valu_summary.py,
# pmc_mfma_summary.py.  A failed step ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
stop() { echo "[profiles] $1 exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
case "${PART:-1}" in
    1)
        ROUND=r05 STEPS=20 WARMUP=5 bash tools/profile_round.sh --no-fitted; stop c3 $?
        ROUND=r05d STEPS=1000 WARMUP=100 bash tools/profile_round.sh --no-fitted; stop c3d $?
        ROUND=r05f STEPS=2 WARMUP=1 bash tools/profile_round.sh; stop c3f $?
        ;;
    2)
        ROUND=r05c5 STEPS=20 WARMUP=5 bash tools/profile_round.sh --workload c5 --no-fitted; stop c5 $?
        ROUND=r05c4 STEPS=1000 WARMUP=100 bash tools/profile_round.sh --workload c4; stop c4 $?
        ROUND=r05c2 STEPS=1000 WARMUP=100 bash tools/profile_round.sh --workload c2 --no-fitted; stop c2 $?
        ;;
    3)
        ROUND=r05 bash tools/pmc_valu.sh; stop valu $?
        ROUND=r05 bash tools/pmc_mfma.sh; stop mfma $?
        ;;
esac
echo "[profiles] part ${PART:-1} done"

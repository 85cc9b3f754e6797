#!/bin/bash
# Round-4 final session 3: the round profiles (C3 at the driver's settings, C5) and the VALU
# PMC passes behind the lambda roofline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
ROUND=r04 bash tools/profile_round.sh
stop prof_c3 $?
ROUND=r04c5 bash tools/profile_round.sh --workload c5
stop prof_c5 $?
bash tools/pmc_valu.sh
stop pmc_valu $?
echo "[session] done"

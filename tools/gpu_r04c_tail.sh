#!/bin/bash
# The measurement tail of GPU sessions c/d: VALU PMC passes, round profiles (C3, C5), bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
bash tools/pmc_valu.sh
stop pmc_valu $?
ROUND=r04 bash tools/profile_round.sh --no-fitted
stop prof_c3 $?
ROUND=r04c5 bash tools/profile_round.sh --workload c5 --no-fitted
stop prof_c5 $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04c_bench_c3d.json 2> gpurun_out/r04c_bench_c3d.err
stop bench $?
python3 -c "
import json; d=json.loads(open('gpurun_out/r04c_bench_c3d.json').read().strip().splitlines()[-1])
print(round(d['value'],1), d['roofline'].get('kernel'), d['roofline'].get('frac'), (d.get('fitted_regime') or {}).get('value'))"
echo "[session] done"

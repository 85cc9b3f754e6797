#!/bin/bash
# Round-4 final session 2: the round's bench lines with CPU baselines and the fitted-regime
# run -- C3 at the driver's settings and at the bench defaults, C1, C2, C4, C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[session] $1 exit $2"; if [ "$2" -ge 124 ] || [ "$2" -eq 134 ] || [ "$2" -eq 139 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench_c3_driver.json 2>> gpurun_out/r04F_bench.err
stop c3_driver $?
timeout -k 10 600 python -u bench.py > gpurun_out/r04_bench_c3.json 2>> gpurun_out/r04F_bench.err
stop c3 $?
for w in c1 c2 c4 c5; do
    case $w in c5) extra="--steps 200 --warmup 20" ;; c1) extra="--steps 20000 --warmup 2000" ;; *) extra="" ;; esac
    timeout -k 10 600 python -u bench.py --workload $w $extra > gpurun_out/r04_bench_$w.json 2>> gpurun_out/r04F_bench.err
    stop $w $?
done
python3 - <<'PY'
import json
for w in ["c3_driver", "c3", "c1", "c2", "c4", "c5"]:
    try:
        d = json.loads(open(f"gpurun_out/r04_bench_{w}.json").read().strip().splitlines()[-1])
    except Exception as ex:
        print(w, "no line", ex)
        continue
    fr = d.get("fitted_regime") or {}
    print(w, round(d["value"], 1), d["roofline"].get("kernel"), d["roofline"].get("frac"),
          (d.get("cpu_baseline") or {}).get("value"), fr.get("value"))
PY
echo "[session] done"

#!/bin/bash
# GPU session: the backward solve's tagged-word hand-off (bb_set_tuning key 20) -- its parity
# test (unless SKIPT), then C4 A/B (300 sweeps after 30) over the --tuning settings in MODES
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$SKIPT" ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    ${TESTS:-tests/test_bsolve_ll_gpu.py tests/test_logit_gpu.py} > gpurun_out/ll_test.log 2>&1
  rc=$?; tail -5 gpurun_out/ll_test.log; [ $rc -ne 0 ] && exit $rc
fi
i=0
for m in ${MODES:-20=1 20=0 20=1 20=0}; do
  i=$((i+1)); f=gpurun_out/ll_b${i}_${m//[=,]/_}
  timeout -k 10 300 python -u bench.py --workload ${WL:-c4} --steps 300 --warmup 30 --no-cpu-baseline --no-fitted --tuning $m > $f.json 2> $f.err || exit 1
  python -c "import json;d=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]);print('$m', round(d['value'],1), round(d['ms_per_step'],4), d['phases_ms'])"
done

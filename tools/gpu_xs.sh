# GPU session: the split lambda launch (bb_set_tuning key 7 = 3) -- its parity tests (unless
# SKIPT is set), then a C3 driver-window A/B over the bench.py --tuning settings in MODES
# (default: key 7 = 3 against 2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$SKIPT" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    ${TESTS:-tests/test_nid_fold_gpu.py tests/test_nid_gpu.py tests/test_shard_nid_gpu.py tests/test_steady_state_gpu.py tests/test_lambda_occ_gpu.py} > gpurun_out/xs_test.log 2>&1
  rc=$?; tail -5 gpurun_out/xs_test.log; [ $rc -ne 0 ] && exit $rc
fi
i=0
for m in ${MODES:-7=3 7=2 7=3 7=2}; do
  i=$((i+1)); f=gpurun_out/xs_b${i}_${m//[=,]/_}
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fitted --tuning $m > $f.json 2> $f.err || exit 1
  python -c "import json;d=json.load(open('$f.json'));r=d['roofline'];print('$m', round(d['value'],1), r['kernel'], round(r['kernel_ms_avg']*1e3,1), d['phases_ms'])"
done

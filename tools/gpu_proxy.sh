# GPU session: the near-identity decision parity tests (unless SKIPT is set), then the per-rank
# proxy of a C3 rank at N = 8 (bench.py --cols 6250, BB_FORCE_RCCL=1, forced K = 2: DESIGN.md
# s7) over the bench.py --tuning settings in MODES
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$SKIPT" ]; then
  timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    ${TESTS:-tests/test_nid_fold_gpu.py tests/test_nid_gpu.py tests/test_shard_nid_gpu.py tests/test_shard8_gpu.py} > gpurun_out/px_test.log 2>&1
  rc=$?; tail -5 gpurun_out/px_test.log; [ $rc -ne 0 ] && exit $rc
fi
i=0
for m in ${MODES:-18=1 18=0 18=1 18=0}; do
  i=$((i+1)); f=gpurun_out/px_b${i}_${m//[=,]/_}
  BB_FORCE_RCCL=1 timeout -k 10 200 python -u bench.py --cols 6250 --steps 20 --warmup 5 --no-cpu-baseline --no-fitted --tuning 16=2 --tuning $m > $f.json 2> $f.err || exit 1
  python -c "import json;d=json.loads([l for l in open('$f.json') if l.startswith('{')][-1]);print('$m', round(d['value'],1), round(d['ms_per_step'],4), d['phases_ms'])"
done

#!/bin/bash
# Which rocprofv3 VALU class counts each instruction of tools/valu_rate (and at what issue
# cost): the microbenchmark once for its cycle table, then once per class counter in its own
# --pmc pass (no trace domain).  Summary: python tools/pmc_valu_summary.py --classes <round>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
ROUND=${ROUND:-r05}
OUT=gpurun_out/valu_classes_$ROUND
mkdir -p "$OUT"
# the sources this profile measures (bench.py uses a profile only for the same tree)
python3 -c "from bayesbridge_amd._build import source_sha; print(source_sha())" > "$OUT/source_sha.txt"
timeout -k 10 120 ./tools/valu_rate 2048 > "$OUT/rates.txt" 2>&1 || { echo "valu_rate failed ($?)"; exit 1; }
echo "rates ok"
for ctr in SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 \
    SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
    SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT; do
    timeout -s KILL 90 rocprofv3 --pmc "$ctr" -d "$OUT/$ctr" -o run --output-format csv \
        -- ./tools/valu_rate 64 > "$OUT/$ctr.log" 2>&1 || { echo "$ctr failed ($?)"; exit 1; }
    echo "$ctr ok"
done

#!/bin/bash
# VALU evidence for the tilted-stable lambda launch ("lambda-step: VALU /
# transcendental ... report draws/s and VALU-busy"): one counter per rocprofv3 --pmc pass
# (no trace domain combined), bench C3 (k_lambda_spec) and C5 (k_lambda_cb), plus the
# near-identity pass k_eapply for reference.  Summary: python tools/pmc_valu_summary.py <round>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
ROUND=${ROUND:-r05}
OUT=gpurun_out/pmc_valu_$ROUND
mkdir -p "$OUT"
# the sources this profile measures (bench.py uses a profile only for the same tree)
python3 -c "from bayesbridge_amd._build import source_sha; print(source_sha())" > "$OUT/source_sha.txt"
# and the code identity of every kernel in the library it runs (bayesbridge_amd/_kernel_code.py)
python3 -m bayesbridge_amd._kernel_code > "$OUT/kernel_code.json" || exit 1
REGEX="k_lambda|k_eapply"
pass() {  # $1 = config name, $2 = counter, rest = bench args
    local cfg=$1 ctr=$2; shift 2
    timeout -s KILL 240 rocprofv3 --pmc "$ctr" --kernel-include-regex "$REGEX" \
        -d "$OUT/$cfg/$ctr" -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline --no-fitted "$@" \
        > "$OUT/$cfg/$ctr.json" 2> "$OUT/$cfg/$ctr.err" || { echo "$cfg $ctr failed ($?)"; exit 1; }
    echo "$cfg $ctr ok"
}
for cfg in ${CONFIGS:-c3 c5}; do
    mkdir -p "$OUT/$cfg"
    case $cfg in
        # the windows of the committed bench lines: C3 the driver's 20 after 5, C5 200 after 20
        c3) args="--steps 20 --warmup 5" ;;
        c5) args="--workload c5 --steps 200 --warmup 20" ;;
    esac
    # the totals, then the per-class counts that price the instructions in SIMD issue cycles
    # (classes and costs: tools/valu_rate.hip, tools/pmc_valu_classes.sh)
    # (COUNTERS=<one counter> runs that pass alone: one GPU step per call)
    for ctr in ${COUNTERS:-SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F64 \
        SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 \
        SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 \
        SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT}; do
        pass $cfg $ctr $args
    done
done

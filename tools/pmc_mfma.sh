#!/bin/bash
# MFMA-busy evidence (north_star): SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE, each in its
# own rocprofv3 --pmc pass (no trace domain combined), over the bench command, for the Gram
# kernels and the Cholesky:
#   c3      default C3 bench (Ozaki-II: k_oz_gemm16u, k_oz_residues; k_chol_persistent)
#   c3fp64  C3 with the fp64 MFMA Gram (k_gram)
#   c2      C2 (k_chol_persistent at n = 1000, k_oz_gemm16u)
#   c4      C4, the logistic bridge (X'OmegaX on k_oz_gemm16u, k_chol_persistent at p = 1000)
# CONFIGS / COUNTERS select configs and counters (one pass per GPU call: COUNTERS=<one>)
# Summary: python tools/pmc_mfma_summary.py <round>  ->  profiles/<round>_pmc_mfma.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
ROUND=${ROUND:-r05}
OUT=gpurun_out/pmc_mfma_$ROUND
mkdir -p "$OUT"
# the sources this profile measures (bench.py uses a profile only for the same tree)
python3 -c "from bayesbridge_amd._build import source_sha; print(source_sha())" > "$OUT/source_sha.txt"
# and the code identity of every kernel in the library it runs (bayesbridge_amd/_kernel_code.py)
python3 -m bayesbridge_amd._kernel_code > "$OUT/kernel_code.json" || exit 1
REGEX="k_oz_gemm16u|k_oz_residues|k_chol_persistent|k_gram"
pass() {  # $1 = config name, $2 = counter, rest = bench args
    local cfg=$1 ctr=$2; shift 2
    timeout -s KILL 240 rocprofv3 --pmc "$ctr" --kernel-include-regex "$REGEX" \
        -d "$OUT/$cfg/$ctr" -o run --output-format csv \
        -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" \
        > "$OUT/$cfg/$ctr.json" 2> "$OUT/$cfg/$ctr.err" || { echo "$cfg $ctr failed ($?)"; exit 1; }
    echo "$cfg $ctr ok"
}
for cfg in ${CONFIGS:-c3 c3fp64 c2 c4}; do
    mkdir -p "$OUT/$cfg"
    case $cfg in
        c3) args="" ;;
        c3fp64) args="--gram fp64" ;;
        c2) args="--workload c2" ;;
        c4) args="--workload c4" ;;
    esac
    for ctr in ${COUNTERS:-SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES}; do
        pass $cfg $ctr $args
    done
done

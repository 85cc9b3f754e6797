#!/bin/bash
# PMC passes on the Ozaki GEMM (each counter group in its own pass; kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc_gemm
mkdir -p $OUT
run() {  # $1 = name, rest = counters
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "k_oz_gemm|k_oz_residues" \
        -d $OUT/$name -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 \
        --gram ozaki --no-cpu-baseline > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; exit 1; }
    echo "$name ok"
}
run tcc TCC_HIT_sum TCC_MISS_sum
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS
run fetch FETCH_SIZE
run grbm GRBM_GUI_ACTIVE GRBM_COUNT

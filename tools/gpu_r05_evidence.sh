#!/bin/bash
# Round-5 evidence steps that run on the GPU box (each under its own limit; a fault, abort or
# timeout ends the script): the published protocol on the four offline rows with ESR (GPU
# chains and the compiled 1-core CPU chain), then the reference-literal p x p sweep at C3 on
# the box's host.  A heartbeat keeps the long single-call CPU steps visibly alive.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 30; do echo "[heartbeat] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
stop() { echo "[evidence] $1 exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
if [ "${ESS:-1}" = "1" ]; then
    METHODS=stable,stable_orth CPU_PROTOCOL=1 timeout -k 10 900 python -u tools/published_ess.py \
        gpurun_out/r05_published_ess.json 2> gpurun_out/r05_published_ess.err > gpurun_out/r05_published_ess.out
    stop published_ess $?
fi
if [ "${LITERAL:-1}" = "1" ]; then
    timeout -k 10 900 python -u tools/literal_c3.py --sweeps 2 --out gpurun_out/r05_cpu_literal_c3.json \
        > gpurun_out/r05_literal.out 2> gpurun_out/r05_literal.err
    stop literal_c3 $?
fi
echo "[evidence] done"

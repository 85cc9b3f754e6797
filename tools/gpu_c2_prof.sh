#!/bin/bash
# C2 default-window profile passes (1000 after 100: kernel trace, FETCH_SIZE, WRITE_SIZE; round
# r06zc2), then the C2 bench line that matches its dominant kernel against them
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for p in kt fetch write; do
    ROUND=r06zc2 STEPS=1000 WARMUP=100 PASS=$p bash tools/profile_round.sh --workload c2 --no-fitted || exit 1
done

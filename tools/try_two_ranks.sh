#!/bin/bash
# Two bench ranks on ONE GPU (both LOCAL_RANK devices forced to 0) to see whether RCCL
# accepts it; expected to fail with "duplicate GPU" on stock RCCL.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export HIP_VISIBLE_DEVICES=0
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
    --rows 1000 --cols 5000 > gpurun_out/two_ranks.log 2>&1
echo "two-rank exit $?"
tail -15 gpurun_out/two_ranks.log

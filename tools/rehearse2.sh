#!/bin/bash
# 2 torchrun ranks sharing the box's one GPU (gloo): exercises the multi-rank
# bench path (rank table, max-over-ranks timing, n_gpus = distinct devices)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OAMD_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr=127.0.0.1 --master-port=29531 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/rehearse2.log 2>&1
rc=$?; grep '^{' gpurun_out/rehearse2.log || tail -20 gpurun_out/rehearse2.log; exit $rc

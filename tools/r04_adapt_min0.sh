#!/bin/bash
# Adaptive extra rounds: minimum 0 (no extra round outside the endgame;
# k_tree reports the chains it could not split) vs 1, after the GPU tests;
# ROUNDS interleaved passes on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-amin0}
export OUT=gpurun_out/$N
bash tools/gpu.sh tests || exit 1
COMMON="--steps 20 --warmup 5 --cpu-baseline-moves 0"
for r in $(seq 1 "${ROUNDS:-3}"); do
  bash tools/gpu.sh "bench min0_$r $COMMON --adaptive-min 0" "bench min1_$r $COMMON --adaptive-min 1" || exit 1
done

#!/bin/bash
# Adaptive extra rounds with the endgame predictor (capi.hip
# pick_extra_rounds) against fixed 8 and 16, the bench's default sustained
# record (64 moves) and a 144-move one; ROUNDS interleaved sweeps on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-aab2}
export OUT=gpurun_out/$N
COMMON="--steps 20 --warmup 5 --cpu-baseline-moves 0"
for r in $(seq 1 "${ROUNDS:-2}"); do
  bash tools/gpu.sh "bench adapt_$r $COMMON" "bench fixed16_$r $COMMON --fixed-extra-rounds --chain-cuts 16" \
    "bench fixed8_$r $COMMON --fixed-extra-rounds --chain-cuts 8" || exit 1
done
bash tools/gpu.sh "bench adapt144 $COMMON --sustained-moves 144" \
  "bench fixed16s144 $COMMON --sustained-moves 144 --fixed-extra-rounds --chain-cuts 16" || exit 1

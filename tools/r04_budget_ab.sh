#!/bin/bash
# Chain budget under the adaptive extra rounds (cuts capped at T x steps /
# budget): 4 (default) vs 3 vs 2 vs 1, ROUNDS interleaved passes on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-budget}
export OUT=gpurun_out/$N
COMMON="--steps 20 --warmup 5 --cpu-baseline-moves 0 --sustained-moves 96"
for r in $(seq 1 "${ROUNDS:-2}"); do
  bash tools/gpu.sh "bench b4_$r $COMMON" "bench b3_$r $COMMON --chain-budget 3 --chain-cuts 17" \
    "bench b1_$r $COMMON --chain-budget 1 --chain-cuts 50" \
    "bench b2_$r $COMMON --chain-budget 2 --chain-cuts 25" || exit 1
done

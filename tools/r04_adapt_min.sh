#!/bin/bash
# Adaptive extra rounds: minimum (= margin over the cuts used) 2 vs 1, ROUNDS
# interleaved passes on one box; then 200-step lines with exact and
# round-robin endgames.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-amin}
export OUT=gpurun_out/$N
COMMON="--steps 20 --warmup 5 --cpu-baseline-moves 0"
for r in $(seq 1 "${ROUNDS:-3}"); do
  bash tools/gpu.sh "bench min2_$r $COMMON --adaptive-min 2" "bench min1_$r $COMMON --adaptive-min 1" || exit 1
done
S200="--steps 200 --warmup 5 --cpu-baseline-moves 0 --sustained-moves 0"
bash tools/gpu.sh "bench s200_exact $S200" "bench s200_rr $S200 --round-robin-endgames"

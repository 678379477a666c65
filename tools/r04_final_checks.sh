#!/bin/bash
# Budget 2 + adaptive rounds: the per-search log (OAMD_ADAPT_LOG) over 20 +
# 144 moves, and 200-step lines with exact and round-robin endgames (same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-fchk}
export OUT=gpurun_out/$N
OAMD_ADAPT_LOG=1 bash tools/gpu.sh "bench log --steps 20 --warmup 5 --sustained-moves 144 --cpu-baseline-moves 0" || exit 1
S200="--steps 200 --warmup 5 --cpu-baseline-moves 0 --sustained-moves 0"
bash tools/gpu.sh "bench s200_exact $S200" "bench s200_rr $S200 --round-robin-endgames"

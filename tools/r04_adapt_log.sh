#!/bin/bash
# Per-search demand of the chain splitting (OAMD_ADAPT_LOG: X, the most cuts
# any game used and the fewest empty squares of a root, per search) at a
# constant X = 16 (OAMD_ADAPT_B=16), 20 + 144 moves of the bench's games.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-alog}
export OUT=gpurun_out/$N
OAMD_ADAPT_LOG=1 OAMD_ADAPT_B=16 bash tools/gpu.sh "bench x16 --steps 20 --warmup 5 --sustained-moves 144 --cpu-baseline-moves 0"

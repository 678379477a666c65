#!/bin/bash
# Same-box A/B of prebuilt variants (abv/) on the bench line with its
# sustained sub-record (whole games: endgames, chain splitting, restarts).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-sab}; shift
OUT=gpurun_out/$N ROUNDS=${ROUNDS:-2} bash tools/gpu.sh "benchvar s --steps 20 --warmup 5 --sustained-moves 72 $*"

#!/bin/bash
# Same-box A/B of the extra rounds' ResNet grid (bench --extra-grid), headline + sustained.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-gab}
for r in 1 2; do
  for g in ${GRIDS:-0 128 32}; do
    OUT=$OUT bash tools/gpu.sh "bench g${g}_$r --steps 20 --warmup 5 --sustained-moves 72 --cpu-baseline-moves 0 --extra-grid $g" || exit 1
  done
done

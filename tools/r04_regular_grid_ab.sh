#!/bin/bash
# Same-box A/B: regular rounds' ResNet on the looping kernel with a capped grid (OAMD_REGULAR_GRID).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-rgab}
for r in 1 2; do
  for g in ${GRIDS:-0 512 256}; do
    OAMD_REGULAR_GRID=$g OUT=$OUT bash tools/gpu.sh "bench rg${g}_$r --steps 20 --warmup 5 --sustained-moves 72 --cpu-baseline-moves 0" || exit 1
  done
done

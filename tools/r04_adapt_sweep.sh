#!/bin/bash
# (OAMD_ADAPT_A / _B / _W were policy knobs of an intermediate build; the engine no longer reads them)
# Policy sweep of the adaptive extra-round count (OAMD_ADAPT_A x used +
# OAMD_ADAPT_B, minimum --adaptive-min) against fixed counts, ROUNDS
# interleaved sweeps on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-asweep}
export OUT=gpurun_out/$N
COMMON="--steps 20 --warmup 5 --sustained-moves 72 --cpu-baseline-moves 0"
for r in $(seq 1 "${ROUNDS:-2}"); do
  OAMD_ADAPT_A=1 OAMD_ADAPT_B=2 bash tools/gpu.sh "bench a1b2m2_$r $COMMON" || exit 1
  OAMD_ADAPT_A=2 OAMD_ADAPT_B=2 bash tools/gpu.sh "bench a2b2m2_$r $COMMON" || exit 1
  OAMD_ADAPT_A=1 OAMD_ADAPT_B=4 bash tools/gpu.sh "bench a1b4m2_$r $COMMON" || exit 1
  OAMD_ADAPT_A=2 OAMD_ADAPT_B=4 bash tools/gpu.sh "bench a2b4m4_$r $COMMON --adaptive-min 4" || exit 1
  bash tools/gpu.sh "bench fixed8_$r $COMMON --fixed-extra-rounds --chain-cuts 8" \
    "bench fixed16_$r $COMMON --fixed-extra-rounds --chain-cuts 16" || exit 1
done

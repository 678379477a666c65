#!/bin/bash
# (OAMD_ADAPT_A / _B / _W were policy knobs of an intermediate build; the engine no longer reads them)
# Adaptive extra rounds, second sweep: X = the most demand (cuts used; 2X when
# a search used all X) over the last OAMD_ADAPT_W measured searches +
# OAMD_ADAPT_B, against the fixed counts; ROUNDS interleaved sweeps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-asweep2}
export OUT=gpurun_out/$N
COMMON="--steps 20 --warmup 5 --sustained-moves 72 --cpu-baseline-moves 0"
for r in $(seq 1 "${ROUNDS:-2}"); do
  OAMD_ADAPT_W=1 OAMD_ADAPT_B=2 bash tools/gpu.sh "bench w1b2_$r $COMMON" || exit 1
  OAMD_ADAPT_W=4 OAMD_ADAPT_B=2 bash tools/gpu.sh "bench w4b2_$r $COMMON" || exit 1
  OAMD_ADAPT_W=8 OAMD_ADAPT_B=2 bash tools/gpu.sh "bench w8b2_$r $COMMON" || exit 1
  OAMD_ADAPT_W=16 OAMD_ADAPT_B=2 bash tools/gpu.sh "bench w16b2_$r $COMMON" || exit 1
  OAMD_ADAPT_W=8 OAMD_ADAPT_B=4 bash tools/gpu.sh "bench w8b4_$r $COMMON" || exit 1
  bash tools/gpu.sh "bench fixed16_$r $COMMON --fixed-extra-rounds --chain-cuts 16" || exit 1
done

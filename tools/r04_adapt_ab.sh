#!/bin/bash
# Adaptive extra rounds (capi.hip pick_extra_rounds): the GPU tests that cover
# them, then same-box bench lines (sustained sub-record included) of the fixed
# count (round-4 default, 8) against the adaptive one, ROUNDS interleaved sweeps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-adapt}
export OUT=gpurun_out/$N
COMMON="--steps 20 --warmup 5 --sustained-moves 72 --cpu-baseline-moves 0"
bash tools/gpu.sh "tests" || exit 1
for r in $(seq 1 "${ROUNDS:-2}"); do
  bash tools/gpu.sh "bench fixed8_$r $COMMON --fixed-extra-rounds --chain-cuts 8" \
    "bench ad2c16_$r $COMMON" "bench ad2c8_$r $COMMON --chain-cuts 8" || exit 1
done

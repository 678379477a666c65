#!/bin/bash
# Chain-splitting sweep (budget, cuts) on the bench line + sustained record, one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-sweep}
DEF="4,6 2,8 2,12 1,16 3,10 4,10 8,3"
for bc in ${SWEEP:-$DEF}; do
  b=${bc%,*}; c=${bc#*,}
  OUT=$OUT bash tools/gpu.sh "bench b${b}c${c} --steps 20 --warmup 5 --sustained-moves 72 --cpu-baseline-moves 0 --chain-budget $b --chain-cuts $c" || exit 1
done

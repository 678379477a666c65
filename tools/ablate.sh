#!/bin/bash
# Build the ablation variants on the box and time each in its own process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OAMD_EXTRA_FLAGS="-DOAMD_ABLATION ${EXTRA:-}" python othello-alphazero_amd/build.py --force > gpurun_out/ablate_build.log 2>&1 || { tail gpurun_out/ablate_build.log; exit 1; }
for v in ${VARIANTS:-0 1 2 4 6 8 9 15}; do
  out=$(OAMD_RESNET_ABLATE=$v timeout -k 10 120 python tools/nn_ablation.py) || { echo "variant $v failed"; exit 1; }
  echo "$out"
done
python othello-alphazero_amd/build.py --force > gpurun_out/ablate_build.log 2>&1

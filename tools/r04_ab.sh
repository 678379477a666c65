#!/bin/bash
# Round-4 A/B of prebuilt variants (abv/, tools/variants.sh): standalone
# ResNet timing (interleaved, outputs compared bit for bit), then the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-ab}
OUT=gpurun_out/$N ROUNDS=3 bash tools/gpu.sh "variants c128" &&
OUT=gpurun_out/$N ROUNDS=3 bash tools/gpu.sh "variants f16 NN_DTYPE=fp16 ROWS=2048" &&
OUT=gpurun_out/$N ROUNDS=2 bash tools/gpu.sh "benchvar c2 --steps 20 --warmup 5 --sustained-moves 0"

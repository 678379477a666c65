#!/bin/bash
# Build liboamd.so variants of the ResNet kernel HERE (CPU container) for the
# GPU-box recipes `variants` / `benchvar` of tools/gpu.sh:
#   VARIANTS="name:extra flags[:path/to/resnet.hip];name2:..." bash tools/variants.sh
# Each variant's resnet.hip (default: the tree's) is compiled with the build's
# flags plus its extra ones and linked with the current tree/capi objects into
# abv/<name>/liboamd.so. Build the default extension first (build.py).
set -eu
cd "$(dirname "$0")/.."
B=othello-alphazero_amd/build
CS=othello-alphazero_amd/csrc
RF="-mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-sched-strategy=max-ilp"
rm -rf abv
IFS=';' read -ra SETS <<< "${VARIANTS:?}"
pids=()
for e in "${SETS[@]}"; do
  IFS=':' read -r name flags src <<< "$e"
  src=${src:-$CS/resnet.hip}
  mkdir -p abv/$name
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $CS -I include -Wall -Wno-unused-function \
      -fno-gpu-rdc $flags $RF -c $src -o abv/$name/resnet.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abv/$name/liboamd.so abv/$name/resnet.o \
      $B/tree.hip.o $B/capi.hip.o && rm abv/$name/resnet.o && echo "built $name" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done

#!/bin/bash
# Build the k_tree phase-stamp diagnostic library (abv/ts/liboamd.so) for
# tools/tree_stamps.py (run on the GPU box by tools/gpu.sh "stamps NAME ts").
set -eu
cd "$(dirname "$0")/.."
CS=othello-alphazero_amd/csrc
CXX="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -fno-gpu-rdc -I $CS -I include -DOAMD_TREE_STAMPS"
EXACT="-ffp-contract=off -fno-fast-math"
NOSCALAR="-mllvm -amdgpu-scalarize-global-loads=false"
RF="-mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-sched-strategy=max-ilp"
mkdir -p abv/ts
$CXX $EXACT $NOSCALAR -c $CS/tree.hip -o abv/ts/tree.o &
$CXX $EXACT -c $CS/capi.hip -o abv/ts/capi.o &
$CXX $RF -c $CS/resnet.hip -o abv/ts/resnet.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abv/ts/liboamd.so abv/ts/*.o
rm -f abv/ts/*.o
echo built abv/ts/liboamd.so

#!/bin/bash
# Build liboamd.so variants HERE (CPU container) for the GPU-box recipes
# `variants` / `benchvar` of tools/gpu.sh:
#   VARIANTS="name:extra flags[:SRC];name2:..." bash tools/variants.sh
# SRC: empty = the tree's resnet.hip with the tree's tree/capi objects; + =
# every unit of the working tree built with the flags;
# a path = that resnet.hip with the tree's tree/capi objects; tree=PATH = that
# tree.hip with the working tree's other units; @REV = all of
# csrc/ and include/ at git revision REV (capi.hip packs the weights, so a
# variant that changes the packing must bring its own capi). Built into
# abv/<name>/liboamd.so (the pybind layer binds the C ABI, not the variant).
set -eu
cd "$(dirname "$0")/.."
B=othello-alphazero_amd/build
CS=othello-alphazero_amd/csrc
RF=${RF-"-mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-sched-strategy=max-ilp"}  # env RF overrides (scheduler A/Bs)
CXX="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -fno-gpu-rdc"
EXACT="-ffp-contract=off -fno-fast-math"
NOSCALAR="-mllvm -amdgpu-scalarize-global-loads=false"  # as build.py builds tree.hip
rm -rf abv
IFS=';' read -ra SETS <<< "${VARIANTS:?}"
pids=()
for e in "${SETS[@]}"; do
  IFS=':' read -r name flags src <<< "$e"
  mkdir -p abv/$name
  (
    set -e
    if [[ "${src:-}" == "+" ]]; then  # every unit of the working tree, built with the flags
      $CXX -I $CS -I include $flags $RF -c $CS/resnet.hip -o abv/$name/resnet.o
      $CXX -I $CS -I include $flags $EXACT $NOSCALAR -c $CS/tree.hip -o abv/$name/tree.o
      $CXX -I $CS -I include $flags $EXACT -c $CS/capi.hip -o abv/$name/capi.o
      objs="abv/$name/tree.o abv/$name/capi.o"
    elif [[ "${src:-}" == tree=* ]]; then  # another tree.hip, the working tree's other units
      $CXX -I $CS -I include $flags $RF -c $CS/resnet.hip -o abv/$name/resnet.o
      $CXX -I $CS -I include $flags $EXACT $NOSCALAR -c ${src#tree=} -o abv/$name/tree.o
      $CXX -I $CS -I include $flags $EXACT -c $CS/capi.hip -o abv/$name/capi.o
      objs="abv/$name/tree.o abv/$name/capi.o"
    elif [[ "${src:-}" == @* ]]; then
      rev=${src#@}; d=abv/$name/src; mkdir -p $d
      git archive "$rev" othello-alphazero_amd/csrc include | tar -x -C $d
      inc="-I $d/$CS -I $d/include"
      $CXX $inc $flags $RF -c $d/$CS/resnet.hip -o abv/$name/resnet.o
      $CXX $inc $EXACT $NOSCALAR -c $d/$CS/tree.hip -o abv/$name/tree.o
      $CXX $inc $EXACT -c $d/$CS/capi.hip -o abv/$name/capi.o
      objs="abv/$name/tree.o abv/$name/capi.o"
    else
      $CXX -I $CS -I include $flags $RF -c ${src:-$CS/resnet.hip} -o abv/$name/resnet.o
      objs="$B/tree.hip.o $B/capi.hip.o"
    fi
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abv/$name/liboamd.so abv/$name/resnet.o $objs
    rm -rf abv/$name/*.o abv/$name/src
    echo "built $name"
  ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done

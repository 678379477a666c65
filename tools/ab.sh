#!/bin/bash
# A/B compile-time variants of the ResNet kernel on the GPU box: for each
# ';'-separated entry of AB, "flags[|dir]", build the extension with those
# flags (and, with |dir, with dir/resnet.hip + dir/capi.hip swapped in) and
# time k_resnet with tools/nn_ablation.py. The default build is restored.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CS=othello-alphazero_amd/csrc
cp $CS/resnet.hip /tmp/resnet.hip.orig && cp $CS/capi.hip /tmp/capi.hip.orig
IFS=';' read -ra SETS <<< "${AB:-}"
for e in "${SETS[@]}"; do
  f="${e%%|*}"; d=""; [[ "$e" == *"|"* ]] && d="${e#*|}"
  if [ -n "$d" ]; then cp "$d/resnet.hip" $CS/resnet.hip && cp "$d/capi.hip" $CS/capi.hip; fi
  rf="-mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-sched-strategy=max-ilp"; [[ "$f" == *NOVGPRFORM* ]] && rf=" "; f="${f//NOVGPRFORM/}"; [[ "$f" == *DEFSCHED* ]] && rf="-mllvm -amdgpu-mfma-vgpr-form=1"; f="${f//DEFSCHED/}"; OAMD_RESNET_FLAGS="$rf" OAMD_EXTRA_FLAGS="$f" python othello-alphazero_amd/build.py --force > gpurun_out/ab_build.log 2>&1 || { echo "build failed: $e"; tail gpurun_out/ab_build.log; exit 1; }
  cp /tmp/resnet.hip.orig $CS/resnet.hip && cp /tmp/capi.hip.orig $CS/capi.hip
  out=$(AB_FLAGS="$f" timeout -k 10 120 python tools/nn_ablation.py) || { echo "timing failed: $e"; exit 1; }
  echo "[$e] $out"
done
python othello-alphazero_amd/build.py --force > gpurun_out/ab_build.log 2>&1

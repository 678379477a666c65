# one A/B batch of ResNet schedule variants (tools/ab.sh), outputs checked bit for bit
cd $GRAFT_REPO_ROOT
export ROWS=4096 AB_REF=/tmp/ab_ref.pt
rm -f $AB_REF
AB="${AB:--DOAMD_BASE=1;-DOAMD_DMA_MODE=1;-DOAMD_DMA_MODE=3;-DOAMD_DMA_MODE=1 -DOAMD_DMA_PIN=4;-DOAMD_DMA_MODE=3 -DOAMD_DMA_PIN=2;-DOAMD_DMA_MODE=3 -DOAMD_DMA_PIN=6;-DOAMD_DMA_MODE=1 -DOAMD_DMA_PIN=7;-DOAMD_BASE=2}" timeout -k 10 1000 bash tools/ab.sh > gpurun_out/ab1.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab1.log; exit $rc

#!/bin/bash
# GPU box: time k_resnet (tools/nn_ablation.py) with each prebuilt variant
# abv/<name>/liboamd.so (tools/build_variants.sh) swapped in, in the order of
# AB_ORDER (default: all, sorted); outputs compared bit for bit with the
# first variant's. ROUNDS > 1 repeats the sweep (interleaved A/B). The
# default liboamd.so is restored at the end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PKG=othello-alphazero_amd/othello_mcts
cp $PKG/liboamd.so /tmp/liboamd.so.orig
export AB_REF=${AB_REF:-/tmp/ab_ref_$$.pt}
rm -f $AB_REF
order=${AB_ORDER:-$(ls abv)}
rc=0
for r in $(seq ${ROUNDS:-1}); do
  for v in $order; do
    cp abv/$v/liboamd.so $PKG/liboamd.so
    out=$(AB_FLAGS="$(cat abv/$v/flags)" timeout -k 10 120 python tools/nn_ablation.py 2>&1 | grep -v amdgpu.ids); rc=$?
    echo "[$v r$r] $out"
    [ $rc -ne 0 ] && break 2
  done
done
cp /tmp/liboamd.so.orig $PKG/liboamd.so
exit $rc

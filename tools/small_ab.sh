#!/bin/bash
# Small-batch ResNet geometry: waves per board (OAMD_SMALL_WC_DIV 4 vs 8) at
# 16 / 32 rows (outputs compared bit for bit), then the single-game latency
# tool for each build. Same box, alternating builds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${DIV_LIST:-4 8 4 8}; do
  OAMD_EXTRA_FLAGS="-DOAMD_SMALL_WC_DIV=$v" python othello-alphazero_amd/build.py --force > gpurun_out/sab_build.log 2>&1 || { tail gpurun_out/sab_build.log; exit 1; }
  for rows in 16 32; do
    out=$(ROWS=$rows AB_REF=/tmp/sab_ref_$rows.pt AB_FLAGS="div=$v" timeout -k 10 120 python tools/nn_ablation.py) || { echo "timing failed: $v"; exit 1; }
    echo "[div=$v rows=$rows] $out"
  done
  timeout -k 10 300 python tools/latency.py > gpurun_out/sab_lat_$v.log 2>&1 || { tail -3 gpurun_out/sab_lat_$v.log; exit 1; }
  grep '^{' gpurun_out/sab_lat_$v.log | sed "s/^/  div=$v /"
done
python othello-alphazero_amd/build.py --force > gpurun_out/sab_build.log 2>&1

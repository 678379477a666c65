#!/bin/bash
# Persistent k_resnet workgroups (OAMD_PERSIST) on/off: kernel timing with
# outputs compared bit for bit (tools/nn_ablation.py, fp32 input) and the
# default bench (packed input), same box, alternating builds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export ROWS=4096 AB_REF=/tmp/ab_ref.pt
rm -f $AB_REF
for v in ${PERSIST_LIST:-0 1 0 1}; do
  OAMD_EXTRA_FLAGS="-DOAMD_PERSIST=$v" python othello-alphazero_amd/build.py --force > gpurun_out/pab_build.log 2>&1 || { tail gpurun_out/pab_build.log; exit 1; }
  out=$(AB_FLAGS="-DOAMD_PERSIST=$v" timeout -k 10 120 python tools/nn_ablation.py) || { echo "timing failed: $v"; exit 1; }
  echo "[persist=$v] $out"
  timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --steps ${STEPS:-10} > gpurun_out/pab_$v.log 2>&1 || { tail -5 gpurun_out/pab_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/pab_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("  bench persist", sys.argv[1], d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], flush=True)
PY
done
python othello-alphazero_amd/build.py --force > gpurun_out/pab_build.log 2>&1

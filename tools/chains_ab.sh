#!/bin/bash
# bench: pipeline groups x NN chains, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${CFGS:-2:1 4:2 4:1 2:1 4:2 3:3}; do
  p=${cfg%%:*}; c=${cfg##*:}
  timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --pipeline $p --nn-chains $c > gpurun_out/ch_${p}_${c}.log 2>&1 || { tail -5 gpurun_out/ch_${p}_${c}.log; exit 1; }
  python3 - "gpurun_out/ch_${p}_${c}.log" "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("groups:chains", sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["rows_per_launch"])
PY
done

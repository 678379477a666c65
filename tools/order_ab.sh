#!/bin/bash
# bench with the NN launches of the two pipeline groups serialised by a token
# event (OAMD_NN_ORDER=1, default) vs unordered (0), same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for o in 1 0 1 0; do
  OAMD_EXTRA_FLAGS="-DOAMD_NN_ORDER=$o" python othello-alphazero_amd/build.py --force > gpurun_out/ob.log 2>&1 || { tail gpurun_out/ob.log; exit 1; }
  timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 > gpurun_out/ord_$o.log 2>&1 || { tail -5 gpurun_out/ord_$o.log; exit 1; }
  python3 - "$o" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ord_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("order", sys.argv[1], d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"])
PY
done
python othello-alphazero_amd/build.py --force > gpurun_out/ob.log 2>&1

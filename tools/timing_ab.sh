#!/bin/bash
# bench value with HIP-event timing on every search vs every 5th (same box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for t in ${EVERY:-1 5 1 5}; do
  timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --timing-every $t > gpurun_out/tab_$t.log 2>&1 || { tail -5 gpurun_out/tab_$t.log; exit 1; }
  python3 - "$t" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/tab_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("every", sys.argv[1], d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"])
PY
done

#!/bin/bash
# bench with the pipeline groups' streams prioritised (OAMD_NN_PRIO: 0 = default
# token ordering, 1 = group 0 high / group 1 low priority and only group 0 waits
# for the token, 2 = prioritised without tokens), same box, same build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python3 -c "import torch; from torch.cuda import Stream; print('priority range', torch.cuda.Stream.priority_range())" || true
for o in ${PRIO_LIST:-0 1 2 0 1 2}; do
  OAMD_NN_PRIO=$o timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --steps ${STEPS:-10} > gpurun_out/prio_$o.log 2>&1 || { tail -5 gpurun_out/prio_$o.log; exit 1; }
  python3 - "$o" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/prio_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("prio", sys.argv[1], d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], flush=True)
PY
done

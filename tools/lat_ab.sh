#!/bin/bash
# Single-game latency (tools/latency.py) for ';'-separated extra build flags
# (OAMD_EXTRA_FLAGS, all units), same box, one build per entry.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${LAT_FLAGS:-}"
i=0
for f in "${SETS[@]}"; do
  i=$((i+1))
  OAMD_EXTRA_FLAGS="$f" python othello-alphazero_amd/build.py --force > gpurun_out/lab_build.log 2>&1 || { tail gpurun_out/lab_build.log; exit 1; }
  timeout -k 10 300 python tools/latency.py > gpurun_out/lab_$i.log 2>&1 || { tail -3 gpurun_out/lab_$i.log; exit 1; }
  grep '^{' gpurun_out/lab_$i.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('[$f]', d['setting'], d.get('median_ms', d.get('wall_ms_per_move')), d.get('tree_us_per_launch',''), d.get('nn_us_per_launch',''), flush=True)"
done
python othello-alphazero_amd/build.py --force > gpurun_out/lab_build.log 2>&1

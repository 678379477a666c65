#!/bin/bash
# Bench (configs[1], no CPU baseline) for ';'-separated extra build flags
# (OAMD_EXTRA_FLAGS), same box, one build per entry.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${BENCH_FLAGS:-}"
i=0
for f in "${SETS[@]}"; do
  i=$((i+1))
  OAMD_EXTRA_FLAGS="$f" python othello-alphazero_amd/build.py --force > gpurun_out/bab_build.log 2>&1 || { tail gpurun_out/bab_build.log; exit 1; }
  timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --steps ${STEPS:-10} ${BENCH_EXTRA:-} > gpurun_out/bab_$i.log 2>&1 || { tail -5 gpurun_out/bab_$i.log; exit 1; }
  python3 - "$i" "$f" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bab_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(f"[{sys.argv[2]}]", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["tree_kernels"]["k_tree"]["avg_launch_ms"], flush=True)
PY
done
python othello-alphazero_amd/build.py --force > gpurun_out/bab_build.log 2>&1

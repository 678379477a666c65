#!/bin/bash
# Bench the single-GPU shapes of BASELINE.json's other configs (short runs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name, args
  timeout -k 10 600 python bench.py --cpu-baseline-seconds 0 "${@:2}" > gpurun_out/cfg_$1.log 2>&1
  rc=$?; echo "== $1 rc=$rc: $(grep '^{' gpurun_out/cfg_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], "sims/s", d["ms_per_step"], "ms/step", r["achieved"], "TF", r["rows_per_launch"], "rows/launch", r["avg_launch_ms"], "ms/launch")' 2>/dev/null)"
  case $rc in 0|1) ;; *) exit $rc ;; esac
}
run c2 --steps 5 --warmup 1
run c4 --steps 2 --warmup 1 --channels 256 --blocks 20 --hidden 256 --sims 1600
run c5 --steps 3 --warmup 1 --games 512 --dtype fp16 --eval-batch 2048
run c5_8k --steps 3 --warmup 1 --games 512 --dtype fp16

#!/bin/bash
# GPU box: bench.py (configs[1], no CPU baseline) with each prebuilt variant
# abv/<name>/liboamd.so (tools/build_variants.sh) swapped in, ROUNDS
# interleaved sweeps; prints value, ms/step and k_resnet ms/launch per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PKG=othello-alphazero_amd/othello_mcts
cp $PKG/liboamd.so /tmp/liboamd.so.orig
rc=0
for r in $(seq ${ROUNDS:-2}); do
  for v in ${AB_ORDER:-$(ls abv)}; do
    cp abv/$v/liboamd.so $PKG/liboamd.so
    timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --steps ${STEPS:-10} ${BENCH_EXTRA:-} > gpurun_out/babp_${v}_$r.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { tail -5 gpurun_out/babp_${v}_$r.log; break 2; }
    python3 - "$v" "$r" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/babp_{sys.argv[1]}_{sys.argv[2]}.log").read().strip().splitlines()[-1])
print(f"[{sys.argv[1]} r{sys.argv[2]}]", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], flush=True)
PY
  done
done
cp /tmp/liboamd.so.orig $PKG/liboamd.so
exit $rc

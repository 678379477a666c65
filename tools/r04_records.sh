#!/bin/bash
# Round-4 record set: GPU tests, the default bench line (+ sustained), kernel
# traces of C2 (20 steps + sustained), C2 200 steps, C4 and C5 for the
# roofline cross-check (tools/prof_summary.py trace), one RCCL-launched line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-rec}
C4="--sims 1600 --channels 256 --blocks 20 --steps 4 --warmup 1 --sustained-moves 0 --cpu-baseline-moves 0"
C5="--games 512 --dtype fp16 --eval-batch 2048 --steps 10 --warmup 2 --sustained-moves 0 --cpu-baseline-moves 0"
OUT=gpurun_out/$N bash tools/gpu.sh tests "bench c2 --steps 20 --warmup 5" \
  "trace c2 --steps 20 --warmup 5 --cpu-baseline-moves 0" \
  "trace s200 --steps 200 --warmup 5 --cpu-baseline-moves 0 --sustained-moves 0" \
  "trace c4 $C4" "trace c5 $C5" \
  "launch c2 --steps 20 --warmup 5 --cpu-baseline-moves 0"

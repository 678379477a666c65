#!/bin/bash
# PMC passes over the configs[1] bench command (one rocprofv3 --pmc pass per
# counter group, each its own run), summarised in the build container by
#   python tools/prof_summary.py bench gpurun_out/<N> c2 <tag>
# -> profiles/<tag>_bench_pmc.json, profiles/traffic_resnet.json and
#    profiles/traffic_tree.json (keyed by kernel-source hash).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-pmc}
A="--steps 20 --warmup 5 --sustained-moves 0 --cpu-baseline-moves 0"
OUT=gpurun_out/$N bash tools/gpu.sh \
  "pmc c2_a SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_INSTS_SALU $A" \
  "pmc c2_b SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU,GRBM_GUI_ACTIVE $A" \
  "pmc c2_c FETCH_SIZE $A" \
  "pmc c2_d WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum $A"

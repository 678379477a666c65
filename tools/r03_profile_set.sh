#!/bin/bash
# Round-3 PMC set of the standalone ResNet kernel for one configuration:
#   bash tools/r03_profile_set.sh PREFIX VAR=val ...   (e.g. c256 NN_C=256)
# four rocprofv3 --pmc passes (SQ wave states / instruction mix, MFMA busy +
# clock + LDS, FETCH_SIZE, WRITE_SIZE + L2 hit), summarised here afterwards by
# python tools/prof_summary.py nn gpurun_out/<OUT> PREFIX <tag>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
p=$1; shift
bash tools/gpu.sh \
  "nnpmc ${p}_a SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_INSTS_SALU $*" \
  "nnpmc ${p}_b SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU,GRBM_GUI_ACTIVE $*" \
  "nnpmc ${p}_c FETCH_SIZE $*" \
  "nnpmc ${p}_d WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum $*"

#!/bin/bash
# One GPU-box records pass for the current build (all raw output under
# gpurun_out/, summarised here afterwards by tools/summarize_prof.py,
# tools/mfma_summary.py and tools/sq_summary.py): rocprofv3 kernel trace +
# stats and FETCH/WRITE passes of the default bench, MFMA busy + clock of the
# bench workload, SQ wave-state counters of k_resnet (standalone), bench lines
# of the other single-GPU configs, single-game latency, and the default bench
# with its CPU baseline. Every step time-limited; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile.sh || exit $?
MFMA_TAG=${TAG:-rec} bash tools/mfma_pmc.sh || exit $?
ROWS=4096 NN_PMC_4="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" bash tools/nn_pmc.sh || exit $?
bash tools/configs.sh || exit $?
timeout -k 10 600 python tools/latency.py > gpurun_out/latency.log 2>&1; rc=$?; echo "== latency rc=$rc"; grep '^{' gpurun_out/latency.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-baseline-seconds 2 > gpurun_out/bench_default.log 2>&1; rc=$?; echo "== bench rc=$rc"; tail -1 gpurun_out/bench_default.log
exit $rc

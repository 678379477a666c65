#!/bin/bash
# MFMA utilisation and the clock the chip holds, for the bench workload:
# one rocprofv3 --pmc pass (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE, with the
# kernel trace for per-dispatch durations), summarised by tools/mfma_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/mfma
mkdir -p $OUT
ARGS="${PROF_BENCH_ARGS:---steps 2 --warmup 1 --cpu-baseline-seconds 0}"
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace \
  -d $OUT/pmc -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc.log 2>&1
rc=$?; echo "== mfma pmc rc=$rc"; tail -2 $OUT/pmc.log
[ $rc -eq 0 ] || exit $rc
python3 tools/mfma_summary.py ${MFMA_TAG:-r01_v7} ${PROF_BENCH_ARGS:+--args "$PROF_BENCH_ARGS"}

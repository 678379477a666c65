#!/bin/bash
# rocprofv3 passes over a short bench run (kernel trace + stats, then one PMC
# counter per pass: FETCH_SIZE and WRITE_SIZE need separate passes on gfx950).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="${PROF_BENCH_ARGS:---steps 2 --warmup 1 --cpu-baseline-seconds 0}"
fatal() { case "$1" in 0|1|2) return 1 ;; *) return 0 ;; esac; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "== trace rc=$rc"; tail -3 $OUT/trace.log; if fatal $rc; then exit $rc; fi
for c in ${PMC_SET:-FETCH_SIZE WRITE_SIZE}; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace -T -d $OUT/pmc_$c -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_$c.log 2>&1
  rc=$?; echo "== pmc $c rc=$rc"; tail -2 $OUT/pmc_$c.log; if fatal $rc; then exit $rc; fi
done
find $OUT -name "*.csv" | head -20

#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench. Stops at the first step that
# dies from a signal / timeout (fault, abort, hang); ordinary test failures
# (exit 1) do not stop the later steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 0|1|2|3|4|5) return 1 ;; *) return 0 ;; esac; }
STEPS="${STEPS:-tests smoke bench}"
for s in $STEPS; do
  case "$s" in
    tests) timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout 300 ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "== $s rc=$rc"
  case "$s" in tests) tail -40 gpurun_out/pytest_gpu.log ;; smoke) tail -20 gpurun_out/smoke.log ;; bench) tail -20 gpurun_out/bench.log ;; esac
  if fatal $rc; then echo "fatal rc=$rc in $s: stopping"; exit $rc; fi
done

#!/bin/bash
# The GPU-box harness: every measurement of DESIGN.md comes from one of these
# recipes (it replaces round 1/2's one-off A/B scripts). Usage:
#   bash tools/gpu.sh "RECIPE ARGS..." ["RECIPE ARGS..." ...]
# Recipes (NAME names the output under $OUT, default gpurun_out/run):
#   tests [pytest args]            the -m gpu suite                  -> tests.log
#   smoke                          __graft_entry__.smoke()           -> smoke.log
#   bench NAME [bench.py args]     one bench line                    -> bench_NAME.json
#   trace NAME [bench.py args]     rocprofv3 --kernel-trace --stats  -> trace_NAME/
#   launch NAME [bench.py args]    bench.py --gpus 1 under torch.distributed.run (one RCCL rank)
#   pmc NAME C1,C2,.. [bench args] one rocprofv3 --pmc pass (+ kernel trace) over bench.py -> pmc_NAME/
#   nn NAME [VAR=val ...]          standalone k_resnet timing (tools/nn_kernel.py; ROWS, NN_C, NN_DTYPE)
#   nnpmc NAME C1,C2,.. [VAR=val]  one --pmc pass over tools/nn_kernel.py  -> nnpmc_NAME/
#   latency NAME                   single-game latency (tools/latency.py)
#   variants NAME [VAR=val ...]    nn timing of every prebuilt abv/<v>/liboamd.so (tools/variants.sh
#                                  builds them here), ROUNDS interleaved sweeps, outputs compared bit
#                                  for bit with the first variant's
#   stamps NAME VARIANT [VAR=val]  tools/nn_stamps.py with abv/VARIANT (built with -DOAMD_STAMPS)
#   benchvar NAME [bench args]     bench line of every prebuilt variant, ROUNDS interleaved sweeps
#   treestamps NAME [VAR=val]      tools/tree_stamps.py with abv/ts (tools/tree_stamps_build.sh)
# Trace post-processing: tools/kt_gaps.py (gaps between ResNet launches), tools/round_profile.py
# (a step split by round). Every step runs under its own time limit; the first failing step ends the run
# (no retries). Summaries: python tools/prof_summary.py (in the build container).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/run}
mkdir -p "$OUT"
PKG=othello-alphazero_amd/othello_mcts

step() {  # step LIMIT LOG cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  echo "== [$rc] $*"
  tail -2 "$log" | cut -c1-400
  return $rc
}

restore_lib() { [ -f /tmp/liboamd.so.orig ] && cp /tmp/liboamd.so.orig $PKG/liboamd.so; }

run_recipe() {
  local recipe=$1; shift
  case "$recipe" in
    tests) step 600 "$OUT/tests.log" python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" ;;
    smoke) step 300 "$OUT/smoke.log" python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) local n=$1; shift; step 900 "$OUT/bench_$n.json" python bench.py "$@" ;;
    launch) local n=$1; shift
      step 900 "$OUT/launch_$n.json" python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
        --master-addr=127.0.0.1 --master-port=29531 bench.py --gpus 1 "$@" ;;
    trace) local n=$1; shift
      step 600 "$OUT/trace_$n.log" rocprofv3 --kernel-trace --stats -T -d "$OUT/trace_$n" -o run \
        --output-format csv -- python3 bench.py "$@" ;;
    pmc) local n=$1 c=$2; shift 2
      step 300 "$OUT/pmc_$n.log" rocprofv3 --pmc ${c//,/ } --kernel-trace -T -d "$OUT/pmc_$n" -o run \
        --output-format csv -- python3 bench.py "$@" ;;
    nn) local n=$1; shift; step 300 "$OUT/nn_$n.log" env "$@" python tools/nn_kernel.py ;;
    nnpmc) local n=$1 c=$2; shift 2
      step 300 "$OUT/nnpmc_$n.log" env "$@" rocprofv3 --pmc ${c//,/ } --kernel-trace -d "$OUT/nnpmc_$n" \
        -o run --output-format csv -- python3 tools/nn_kernel.py ;;
    latency) step 600 "$OUT/latency_$1.log" python tools/latency.py ;;
    variants) local n=$1; shift
      cp $PKG/liboamd.so /tmp/liboamd.so.orig
      local ref=/tmp/ab_ref_$n.pt; rm -f $ref
      for r in $(seq ${ROUNDS:-2}); do
        for v in ${AB_ORDER:-$(ls abv)}; do
          cp abv/$v/liboamd.so $PKG/liboamd.so
          step 300 "$OUT/var_${n}_${v}_$r.log" env AB_REF=$ref "$@" python tools/nn_kernel.py || { restore_lib; return 1; }
        done
      done
      restore_lib ;;
    stamps) local n=$1 v=$2; shift 2  # tools/nn_stamps.py on a -DOAMD_STAMPS variant
      cp $PKG/liboamd.so /tmp/liboamd.so.orig
      cp abv/$v/liboamd.so $PKG/liboamd.so
      step 300 "$OUT/stamps_$n.log" env "$@" python tools/nn_stamps.py; local rc=$?
      restore_lib; return $rc ;;
    treestamps) local n=$1; shift
      cp $PKG/liboamd.so /tmp/liboamd.so.orig
      cp abv/ts/liboamd.so $PKG/liboamd.so
      step 600 "$OUT/treestamps_$n.log" env "$@" python -u tools/tree_stamps.py; local rc=$?
      restore_lib; return $rc ;;
    benchvar) local n=$1; shift
      cp $PKG/liboamd.so /tmp/liboamd.so.orig
      for r in $(seq ${ROUNDS:-2}); do
        for v in ${AB_ORDER:-$(ls abv)}; do
          cp abv/$v/liboamd.so $PKG/liboamd.so
          step 600 "$OUT/benchvar_${n}_${v}_$r.json" env OAMD_AB_VARIANT=$v python bench.py --cpu-baseline-moves 0 \
            --deep-tree-moves 0 --latency-moves 0 --no-config-records "$@" || { restore_lib; return 1; }
        done
      done
      restore_lib ;;
    *) echo "unknown recipe: $recipe"; return 2 ;;
  esac
}

for s in "$@"; do
  # shellcheck disable=SC2086
  run_recipe $s || exit $?
done

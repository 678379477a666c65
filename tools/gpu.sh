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
#   lattrace NAME SIMS             kernel trace of single-game searches (tools/latency_trace.py; EPS env)
#   stress NAME [MOVES CHUNK]      free-running vs lock step over many game generations (tools/stress_free.py)
#   variants NAME [VAR=val ...]    nn timing of every prebuilt abv/<v>/liboamd.so (tools/variants.sh
#                                  builds them here), ROUNDS interleaved sweeps, outputs compared bit
#                                  for bit with the first variant's
#   stamps NAME VARIANT [VAR=val]  tools/nn_stamps.py with abv/VARIANT (built with -DOAMD_STAMPS)
#   benchvar NAME [bench args]     bench line of every prebuilt variant, ROUNDS interleaved sweeps
#   latvar NAME                    tools/latency.py with every prebuilt variant, ROUNDS sweeps
#   treestamps NAME [VAR=val]      tools/tree_stamps.py with abv/ts (tools/tree_stamps_build.sh)
#   records                        the canonical record set: tests, the C2 bench line (20 + 5 steps), kernel
#                                  traces of C2 / 200 steps / C4 / C5, the C2 line under torch.distributed.run
#                                  (summary: tools/record_summary.py)
#   benchpmc NAME                  the four PMC passes over the C2 bench (tools/prof_summary.py bench)
#   nnpmcset NAME [VAR=val ...]    the four PMC passes over the standalone kernel (tools/prof_summary.py nn)
#   hostcpu NAME                   host CPU per rank: tools/host_threads.py and 2 interleaved short bench
#                                  lines, poll-and-sleep waits vs OAMD_SPIN_SYNC=1 --spin-sync, then the
#                                  world-2 gloo rehearsal on the one GPU (round 6)
#   winoprobe NAME                 the Winograd tower probe and its attribution builds vs NativeNet
#                                  (tools/winograd_probe.py; build: tools/winograd_probe_build.sh)
# A/B sweeps are plain recipe lists, e.g. ROUNDS of
#   bash tools/gpu.sh "bench a_1 ARGS_A" "bench b_1 ARGS_B" "bench a_2 ARGS_A" "bench b_2 ARGS_B"
# (the round-4 one-off sweep scripts were folded into this form; their results are in profiles/r04/ab/).
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
    lattrace) local n=$1 sims=$2  # kernel trace of single-game searches (EPS from the environment)
      step 600 "$OUT/lattrace_$n.log" rocprofv3 --kernel-trace -T -d "$OUT/lattrace_$n" -o run \
        --output-format csv -- python3 tools/latency_trace.py "$sims" ;;
    pmc) local n=$1 c=$2; shift 2
      step 300 "$OUT/pmc_$n.log" rocprofv3 --pmc ${c//,/ } --kernel-trace -T -d "$OUT/pmc_$n" -o run \
        --output-format csv -- python3 bench.py "$@" ;;
    nn) local n=$1; shift; step 300 "$OUT/nn_$n.log" env "$@" python tools/nn_kernel.py ;;
    nnpmc) local n=$1 c=$2; shift 2
      step 300 "$OUT/nnpmc_$n.log" env "$@" rocprofv3 --pmc ${c//,/ } --kernel-trace -d "$OUT/nnpmc_$n" \
        -o run --output-format csv -- python3 tools/nn_kernel.py ;;
    latency) step 600 "$OUT/latency_$1.log" python tools/latency.py ;;
    stress) step 900 "$OUT/stress_$1.log" python -u tools/stress_free.py "${@:2}" ;;
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
            --deep-tree-moves 0 --latency-moves 0 --no-config-records --no-ceiling-probe "$@" || { restore_lib; return 1; }
        done
      done
      restore_lib ;;
    latvar) local n=$1; shift  # tools/latency.py with every prebuilt abv/<v>/liboamd.so
      cp $PKG/liboamd.so /tmp/liboamd.so.orig
      for r in $(seq ${ROUNDS:-2}); do
        for v in ${AB_ORDER:-$(ls abv)}; do
          cp abv/$v/liboamd.so $PKG/liboamd.so
          step 300 "$OUT/latvar_${n}_${v}_$r.log" python tools/latency.py || { restore_lib; return 1; }
        done
      done
      restore_lib ;;
    records)
      local C2="--steps 20 --warmup 5" C4="--sims 1600 --channels 256 --blocks 20 --hidden 256 --steps 4 --warmup 1"
      local C5="--games 512 --dtype fp16 --eval-batch 2048 --steps 10 --warmup 2"
      local Q="--sustained-moves 0 --cpu-baseline-moves 0 --deep-tree-moves 0 --latency-moves 0 --no-config-records --no-ceiling-probe"
      run_recipe tests && run_recipe bench c2 $C2 && run_recipe trace c2 $C2 $Q &&
        run_recipe trace s200 --steps 200 --warmup 5 $Q && run_recipe trace c4 $C4 $Q &&
        run_recipe trace c5 $C5 $Q && run_recipe launch c2 $C2 $Q ;;
    benchpmc) local n=$1
      local A="--steps 20 --warmup 5 --sustained-moves 0 --cpu-baseline-moves 0 --deep-tree-moves 0 --latency-moves 0 --no-config-records"
      run_recipe pmc ${n}_a SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_INSTS_SALU $A &&
        run_recipe pmc ${n}_b SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU,GRBM_GUI_ACTIVE $A &&
        run_recipe pmc ${n}_c FETCH_SIZE $A && run_recipe pmc ${n}_d WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum $A ;;
    nnpmcset) local p=$1; shift
      run_recipe nnpmc ${p}_a SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_INSTS_SALU "$@" &&
        run_recipe nnpmc ${p}_b SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU,GRBM_GUI_ACTIVE "$@" &&
        run_recipe nnpmc ${p}_c FETCH_SIZE "$@" && run_recipe nnpmc ${p}_d WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum "$@" ;;
    hostcpu) local n=$1
      local A="--steps 20 --warmup 5 --sustained-moves 0 --cpu-baseline-moves 0 --deep-tree-moves 0 --latency-moves 0 --no-config-records"
      step 200 "$OUT/hostcpu_${n}_threads_poll.json" python tools/host_threads.py &&
        step 200 "$OUT/hostcpu_${n}_threads_spin.json" env OAMD_SPIN_SYNC=1 python tools/host_threads.py --spin-sync || return 1
      for r in 1 2; do
        step 300 "$OUT/hostcpu_${n}_poll_$r.json" python bench.py $A &&
          step 300 "$OUT/hostcpu_${n}_spin_$r.json" env OAMD_SPIN_SYNC=1 python bench.py $A --spin-sync || return 1
      done
      step 600 "$OUT/hostcpu_${n}_rehearsal_world2_gloo.json" env OAMD_BENCH_BACKEND=gloo python bench.py --gpus 2 $A ;;
    winoprobe) local n=$1 P=tools/_build
      step 300 "$OUT/winoprobe_$n.json" python tools/winograd_probe.py $P/libwinoprobe_q4.so $P/libwinoprobe_noT.so \
        $P/libwinoprobe_noE.so $P/libwinoprobe_noTE.so ;;
    *) echo "unknown recipe: $recipe"; return 2 ;;
  esac
}

for s in "$@"; do
  # shellcheck disable=SC2086
  run_recipe $s || exit $?
done

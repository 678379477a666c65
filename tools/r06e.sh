set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06e; mkdir -p $O
Q="--steps 20 --warmup 5 --sustained-moves 0 --cpu-baseline-moves 0 --deep-tree-moves 0 --latency-moves 0 --no-config-records"
P=tools/_build
timeout -k 10 300 python tools/winograd_probe.py $P/libwinoprobe_q4.so $P/libwinoprobe_noT.so $P/libwinoprobe_noE.so $P/libwinoprobe_noTE.so > $O/winograd_probe.json 2>&1 || exit 1
timeout -k 10 200 python tools/host_threads.py > $O/threads_poll.json 2>&1 || exit 1
OAMD_SPIN_SYNC=1 timeout -k 10 200 python tools/host_threads.py --spin-sync > $O/threads_spin.json 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py $Q > $O/poll_$i.json 2> $O/poll_$i.err || exit 1
  OAMD_SPIN_SYNC=1 timeout -k 10 300 python bench.py $Q --spin-sync > $O/spin_$i.json 2> $O/spin_$i.err || exit 1
done
OAMD_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 $Q > $O/rehearsal_world2_gloo.json 2> $O/rehearsal.err || exit 1
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
echo done

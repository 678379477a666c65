set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06d; mkdir -p $O
Q="--steps 20 --warmup 5 --sustained-moves 0 --cpu-baseline-moves 0 --deep-tree-moves 0 --latency-moves 0 --no-config-records"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python tools/winograd_probe.py tools/_build/libwinoprobe_q4.so tools/_build/libwinoprobe_q8.so > $O/winograd_probe.json 2>&1 || exit 1
timeout -k 10 200 python tools/host_threads.py > $O/threads_blk.json 2>&1 || exit 1
OAMD_SPIN_SYNC=1 timeout -k 10 200 python tools/host_threads.py --spin-sync > $O/threads_spin.json 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py $Q > $O/blk_$i.json 2> $O/blk_$i.err || exit 1
  OAMD_SPIN_SYNC=1 timeout -k 10 300 python bench.py $Q --spin-sync > $O/spin_$i.json 2> $O/spin_$i.err || exit 1
done
echo done

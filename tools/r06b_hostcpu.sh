set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06b; mkdir -p $O
Q="--steps 20 --warmup 5 --sustained-moves 0 --cpu-baseline-moves 0 --deep-tree-moves 0 --latency-moves 0 --no-config-records"
for i in 1 2; do
  timeout -k 10 300 python bench.py $Q > $O/blk_$i.json 2> $O/blk_$i.err || exit 1
  OAMD_SPIN_SYNC=1 timeout -k 10 300 python bench.py $Q --spin-sync > $O/spin_$i.json 2> $O/spin_$i.err || exit 1
done
OAMD_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 $Q > $O/rehearsal_world2_gloo.json 2> $O/rehearsal.err || exit 1
echo done

"""Benchmark: whole-node MCTS simulations/sec, 800 sims/move, 128x10b ResNet.

BASELINE.json metric on configs[1] (256 concurrent self-play games, 128x10b,
bf16, one MI355X) per GPU; with --gpus N (torchrun, one process per GPU) every
rank runs its own 256 games (games shard embarrassingly: no collective on the
hot path, "scaling": "weak").

A step is one self-play move of every game on the GPU: a full 800-simulation
search (25 steps of select -> fused ResNet -> expand/backup for T=2 x B=16
leaves per game) followed by the on-device move choice, 8-fold target emission
and move application (finished games restart from a random opening).
Synthetic data: random-init AlphaZeroNet weights of the 128x10b architecture
(seeded), random openings of 0..8 plies.

Also reported (rank 0):
  roofline      the fused ResNet kernel: algorithmic FLOPs (342.3 MFLOP per
                evaluated leaf) / its average HIP-event duration, vs the
                2.5 PFLOP/s dense bf16 MFMA peak; traffic from profiles/ if a
                PMC summary for this config exists, else null.
  cpu_baseline  the oracle C restatement of the reference search + torch-CPU
                fp32 ResNet, 1 game (configs[0]), bounded sample on this host.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0}  # MI355X dense MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
# BASELINE.md "Published numbers for this path": the reference on 1x RTX 4090 +
# 24-core CPU, 128x10b, history 8, 800 sims/move, 2 threads x 16 (README.md:25)
PUBLISHED_SIMS_PER_S = 28000.0


def resnet_flops_per_eval(in_ch: int, C: int, R: int, hidden: int) -> float:
    conv0 = 2 * 64 * 9 * in_ch * C
    tower = 2 * R * 2 * 64 * 9 * C * C
    heads = 2 * 64 * C * 3 + 2 * 128 * 65 + 2 * 64 * hidden + 2 * hidden
    return float(conv0 + tower + heads)


def cpu_baseline(seconds: float, history: int, C: int, R: int, hidden: int, max_moves: int | None = None,
                 warmup_moves: int = 0) -> dict:
    """Oracle port of the reference CPU path (configs[0]): 1 game, 2 threads x 16,
    800 sims/move, fp32 torch-CPU ResNet; moves until `seconds` elapse (or
    `max_moves`), after `warmup_moves` untimed moves. Validated against the
    compiled reference in the build container: tools/cpu_baseline_validate.py,
    profiles/r02_cpu_baseline_validation.json."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import numpy as np

    import oracle as O
    import resnet_ref
    from othello_mcts.synthetic import alphazero_state_dict

    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in
          alphazero_state_dict(1, 1 + 2 * history, C, R, hidden).items()}

    def nn(feat):
        with torch.no_grad():
            out = resnet_ref.forward(sd, torch.from_numpy(np.ascontiguousarray(feat)))
        return out["policy"].numpy(), out["value"].numpy()

    m = O.OracleMCTS(history_size=history, num_simulations=800, num_threads=2, batch_size=16,
                     dirichlet_epsilon=0.25, game_key=5)
    def move():
        if m.position().player == 0:
            m.reset_position()
        n = m.search(nn)
        vc = m.visit_counts()
        m.apply_action(O.legal_actions(m.position())[int(np.argmax(vc))])
        return n

    for _ in range(warmup_moves):
        move()
    sims = 0
    moves = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds and (max_moves is None or moves < max_moves):
        sims += move()
        moves += 1
    dt = time.perf_counter() - t0
    return {"value": round(sims / dt, 1), "unit": "simulations/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)),
            "sample": f"1 game from the initial position, {moves} moves x 800 sims (T=2 x B=16, "
                      f"eps=0.25), {C}x{R + 1}b fp32 torch-CPU, {dt:.1f} s"}


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ---- multi-GPU plumbing (one process per GPU; games shard, no data-path
# collective). Kept device-agnostic so tests/test_dist_cpu.py runs it with gloo.

def dist_env() -> tuple[int, int, int]:
    """(world, rank, local_rank) from the torchrun environment (1, 0, 0 if unset)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_seeds(seed: int, rank: int) -> tuple[int, int]:
    """Per-rank (engine RNG key, opening seed): every rank plays its own games."""
    return seed + 7919 * rank, seed + rank


def timed_max(world: int, run, sync, device: str) -> float:
    """Run `run()` bracketed by barrier + device sync on both sides; return the
    MAX wall time over ranks (the whole job's time)."""
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    run()
    sync()
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def rank_table(world: int, rank: int, device_id: str, sims: int) -> list[dict]:
    """[{rank, device, sims}] of every rank (all_gather_object over the job's
    process group): which physical device each rank ran on and its units."""
    me = {"rank": rank, "device": device_id, "sims": sims}
    if world == 1:
        return [me]
    out: list = [None] * world
    dist.all_gather_object(out, me)
    return out


def aggregate_rate(world: int, games: int, sims_per_search: int, steps: int, dt_max: float) -> float:
    """Whole-job simulations/s: the units all ranks processed / the max time."""
    return world * games * sims_per_search * steps / dt_max


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--games", type=int, default=256, help="concurrent games per GPU")
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--threads", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--history", type=int, default=8)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--blocks", type=int, default=10, help="conv block + residual blocks")
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--eval-batch", type=int, default=0,
                    help="NN rows per ResNet launch (0 = a whole pipeline group, games*L/2 rows); "
                         "configs[4] uses 2048")
    ap.add_argument("--pipeline", type=int, default=0, help="pipeline groups (0 = engine default: 2)")
    ap.add_argument("--nn-chains", type=int, default=1, help="concurrent chains of ResNet launches")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--seed", type=int, default=2025)
    ap.add_argument("--sync-search", action="store_true", help="host waits for every search (diagnostic)")
    ap.add_argument("--timing-every", type=int, default=5,
                    help="record the kernels' HIP events on every N-th timed search (1 = all; the event "
                         "packets add ~10 us per NN launch boundary to the searches they time)")
    args = ap.parse_args()

    world, rank, local = dist_env()
    # OAMD_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share
    # devices round-robin, timing reduced over gloo); the driver's runs use RCCL
    backend = os.environ.get("OAMD_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import othello_mcts as om
    from othello_mcts.synthetic import alphazero_state_dict

    R = args.blocks - 1
    sd = alphazero_state_dict(args.seed, 1 + 2 * args.history, args.channels, R, args.hidden)
    net = om.NativeNet(sd, device=local, dtype=args.dtype)
    engine_seed, opening_seed = shard_seeds(args.seed, rank)
    b = om.BatchedMCTS(args.games, history_size=args.history, num_simulations=args.sims,
                       num_threads=args.threads, batch_size=args.batch, seed=engine_seed)
    b.random_openings(8, seed=opening_seed)
    L = args.threads * args.batch
    if args.eval_batch:  # rows per ResNet launch; the 2 pipeline groups stay
        b.engine.set_nn_batch(args.eval_batch)
    if args.pipeline:
        b.engine.set_pipeline(args.pipeline)
    b.engine.set_nn_chains(args.nn_chains)
    sims_per_search = L * ((args.sims + L - 1) // L)

    def step():
        b.search(net, sync=args.sync_search)  # enqueue only; the timed region syncs at its end
        b.selfplay_move(temperature_moves=12, opening_moves=8, emit_targets=True)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    b.engine.enable_timing(max(1, args.timing_every))
    ms0, launches0, rows0 = b.engine.nn_timing()
    sel0, bk0, tree_launches0 = b.engine.tree_timing()

    def run():
        for _ in range(args.steps):
            step()

    dt_max = timed_max(world, run, torch.cuda.synchronize, "cpu" if backend == "gloo" else "cuda")
    ms1, launches1, rows1 = b.engine.nn_timing()
    sel1, bk1, tree_launches1 = b.engine.tree_timing()
    value = aggregate_rate(world, args.games, sims_per_search, args.steps, dt_max)
    # every game's search followed the reference: no node pool ran out
    overflow_games, depth_capped = b.engine.status()
    if overflow_games or depth_capped:
        raise SystemExit(f"bench invalid: {overflow_games} game(s) overflowed their node pool, "
                         f"{depth_capped} hit the depth cap")
    props = torch.cuda.get_device_properties(local)
    dev_id = f"{os.uname().nodename}:{getattr(props, 'uuid', local)}"
    ranks = rank_table(world, rank, dev_id, args.games * sims_per_search * args.steps)
    n_devices = len({r["device"] for r in ranks})

    nn_ms = ms1 - ms0
    nn_launches = launches1 - launches0
    nn_rows = rows1 - rows0
    flops = resnet_flops_per_eval(1 + 2 * args.history, args.channels, R, args.hidden)
    avg_ms = nn_ms / max(1, nn_launches)
    rows_per_launch = nn_rows / max(1, nn_launches)
    achieved = flops * rows_per_launch / (avg_ms * 1e-3) / 1e12
    executed = flops - 2.0 * 64 * 9 * args.channels * args.channels * 2 * R // 12
    peak = PEAK_TFLOPS[args.dtype]
    workload = (f"{args.games} concurrent self-play games per GPU, {args.sims} sims/move, "
                f"{args.channels}x{args.blocks}b ResNet {args.dtype}, history {args.history}, "
                f"{args.threads} threads x {args.batch} leaves per step"
                + (f", eval batch {args.eval_batch}" if args.eval_batch else "")
                + (" (BASELINE configs[1])" if (args.games, args.channels, args.blocks, args.sims, args.dtype,
                                                args.eval_batch) == (256, 128, 10, 800, "bf16", 0) else ""))
    # HBM bytes per launch from the committed PMC summary of this same workload
    traffic = None
    tfile = ROOT / "profiles" / "traffic_resnet.json"
    if tfile.exists():
        try:
            tj = json.loads(tfile.read_text())
            if tj.get("workload") == workload and tj.get("rows_per_launch") == int(rows_per_launch):
                traffic = tj.get("bytes_per_launch")
        except (ValueError, OSError):
            traffic = None

    # tree kernels: latency-bound (one wave per game, dependent loads); HBM bytes
    # per launch from the committed PMC summary of this workload, if present
    tree_bytes = {}
    tfile = ROOT / "profiles" / "traffic_tree.json"
    if tfile.exists():
        try:
            tj = json.loads(tfile.read_text())
            if tj.get("workload") == workload and tj.get("rows_per_launch") == int(rows_per_launch):
                tree_bytes = {k: v["bytes_per_launch"] for k, v in tj["kernels"].items()}
        except (ValueError, OSError, KeyError):
            tree_bytes = {}
    # k_tree: one launch per search round and pipeline group; "select" rounds
    # back up the previous batch and select the next, the final round backs up
    tree = {"bound": "latency", "sims_per_launch": int(rows_per_launch)}
    tree_launches = tree_launches1 - tree_launches0  # select rounds x pipeline groups
    steps_per_search = (args.sims + L - 1) // L
    for name, ms, n in (("k_tree", sel1 - sel0, tree_launches),
                        ("k_tree_final_backup", bk1 - bk0, tree_launches // steps_per_search)):
        avg = ms / max(1, n)
        entry = {"avg_launch_ms": round(avg, 4)}
        if name in tree_bytes:
            gbs = tree_bytes[name] / (avg * 1e-3) / 1e9
            entry.update({"hbm_bytes_per_launch": tree_bytes[name], "achieved_GB_s": round(gbs, 2),
                          "frac_hbm_peak": round(gbs / PEAK_HBM_GBS, 5)})
        tree[name] = entry

    result = {
        "metric": "MCTS simulations/sec (whole node), 800 sims/move, 128x10b ResNet, 1/2/4/8 GPU",
        "value": round(value, 1),
        "unit": "simulations/s",
        "n_gpus": n_devices,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt_max * 1e3 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / PUBLISHED_SIMS_PER_S, 2),
        "baseline_ref": {"value": PUBLISHED_SIMS_PER_S, "unit": "simulations/s",
                         "hardware": "1x RTX 4090 + 24-core CPU (reference README.md:25, BASELINE.md)"},
        "dtype": args.dtype,
        "data": f"synthetic: seeded random-init {args.channels}x{args.blocks}b AlphaZeroNet weights, "
                "random openings (0-8 plies)",
        "config": {
            "workload": workload,
            "games_per_gpu": args.games,
            "sims_per_move": args.sims,
            "leaves_per_step": L,
            "parallelism": (f"games sharded over {world} rank(s) on {n_devices} GPU(s), no collective"
                            + (" (REHEARSAL: ranks share GPUs; not a scaling point)"
                               if n_devices < world else "")),
            "ranks": ranks,
            "backend": (backend if world > 1 else "none"),
        },
        "overflow_games": overflow_games,
        "roofline": {
            "bound": "mfma",
            "kernel": "k_resnet_w8 (fused 19-conv tower + heads, 8-wave geometry)",
            "achieved": round(achieved, 2),
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "traffic": traffic,
            "avg_launch_ms": round(avg_ms, 4),
            "rows_per_launch": int(rows_per_launch),
            "flops_per_row": flops,
            # the default build leaves out the tower MFMAs whose activations are
            # all zero border (1/12 of every tower conv): achieved
            # counts the algorithmic FLOPs above, these are the ones executed
            "executed_flops_per_row": executed,
            "executed_TFLOP_s": round(executed * rows_per_launch / (avg_ms * 1e-3) / 1e12, 2),
        },
        "tree_kernels": tree,
    }
    if rank == 0 and world == 1 and args.cpu_baseline_seconds > 0:
        result["cpu_baseline"] = cpu_baseline(args.cpu_baseline_seconds, args.history, args.channels, R,
                                              args.hidden)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Benchmark: whole-node MCTS simulations/sec, 800 sims/move, 128x10b ResNet.

BASELINE.json metric on configs[1] (256 concurrent self-play games, 128x10b,
bf16, one MI355X) per GPU. With --gpus N every rank (one process per GPU)
runs its own 256 games: games shard embarrassingly, no collective on the hot
path, "scaling": "weak". The rank processes come from the driver's
torch.distributed.run, or, when bench.py is started bare with --gpus N > 1,
from a torch.distributed.run child that bench.py starts itself before it
touches the GPU. A run whose ranks do not match --gpus, or whose ranks share
GPUs without the explicit gloo rehearsal (OAMD_BENCH_BACKEND=gloo), fails.

A step is one self-play move of every game on the GPU: a full 800-simulation
search (25 steps of select -> fused ResNet -> expand/backup for T=2 x B=16
leaves per game) followed by the on-device move choice, 8-fold target emission
and move application (finished games restart from a random opening). The K
timed steps are one multi-move call (BatchedMCTS.selfplay_steps: per game the
same kernels in the same order as K search + selfplay_move pairs; each
pipeline group chains its moves on its own stream); --per-move-calls times K
call pairs instead.
Synthetic data: random-init AlphaZeroNet weights of the 128x10b architecture
(seeded), random openings of 0..8 plies.

Also reported (rank 0):
  roofline      the fused ResNet kernel: algorithmic FLOPs (342.3 MFLOP per
                evaluated leaf, n_eval = rows of non-terminal leaves,
                BASELINE.md) / its average HIP-event duration, vs the 2.5
                PFLOP/s dense bf16 MFMA peak; traffic from profiles/ if a PMC
                summary for this config exists, else null.
  cpu_baseline  the oracle C restatement of the reference search + torch-CPU
                fp32 ResNet, 1 game (configs[0]), a fixed number of moves after
                a fixed warm-up, torch threads = the CPUs this process may use.

--dry-run exercises the rank plumbing (launch, checks, barrier-bracketed
max-over-ranks timing, rank table, aggregation, the JSON line) with no GPU and
no search: gloo on the CPU, every step a fixed sleep. Its line says so.
"""

from __future__ import annotations

import argparse
import json
import os
import resource
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "MCTS simulations/sec (whole node), 800 sims/move, 128x10b ResNet, 1/2/4/8 GPU"
PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0}  # MI355X dense MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
# BASELINE.md "Published numbers for this path": the reference on 1x RTX 4090 +
# 24-core CPU, 128x10b, history 8, 800 sims/move, 2 threads x 16 (README.md:25)
PUBLISHED_SIMS_PER_S = 28000.0


def kernel_hash(kind: str) -> str:
    """sha256 (16 hex digits) over the HIP sources of one kernel family, as
    compiled into the LOADED liboamd.so (othello_mcts/provenance.py; the
    committed PMC traffic records profiles/traffic_*.json carry it, a record
    of other code is not used). EngineWorkload first checks that the library
    was built from the sources on disk."""
    from othello_mcts import provenance

    return provenance.loaded_hash(kind)


def pipeline_groups(args) -> int:
    """Pipeline groups of the native search (capi.hip plan_groups)."""
    k = args.pipeline if args.pipeline > 0 else (2 if args.games >= 64 else 1)
    return max(1, min(k, args.games, 8))


def single_game_split(args) -> bool:
    """One game, T > 1: the thread-split schedule (capi.hip oamd_engine_search)."""
    return args.games == 1 and pipeline_groups(args) == 1 and 1 < args.threads <= 8


def max_search_rounds(args) -> int:
    """The most NN rounds one native search runs: one per batch of a thread,
    plus up to chain_cuts extra rounds (exact interleaving only; the engine
    picks each search's count adaptively, capi.hip pick_extra_rounds, and
    reports the rounds it ran: oamd_engine_round_counts)."""
    steps = (args.sims + args.threads * args.batch - 1) // (args.threads * args.batch)
    # (capi.hip extra_rounds: no game can use more cuts than T x steps / budget)
    extra = (min(args.chain_cuts, args.threads * steps // args.chain_budget)
             if (not args.round_robin_endgames and args.chain_budget > 0 and not single_game_split(args)) else 0)
    return steps + extra


# SURVEY.md §8(d) "algorithmic bytes per simulation" of the tree kernels, per
# item: a descent level reads its children's N, W, P (12 B each) and writes the
# virtual loss (16 B RMW), the backup writes each level again (16 B RMW); an
# expansion writes 28 B per created child + an 8 B child-range record; an NN
# row gathers H x 16 B of history, writes (1 + 2H) x 8 B of bit-packed
# features and reads back 65 x 2 + 2 B of policy / value.
TREE_BYTES = {"per_child_scanned": 12, "per_level": 16 + 16, "per_expansion": 8, "per_child_created": 28}


def tree_bytes_per_row(history: int) -> int:
    return history * 16 + (1 + 2 * history) * 8 + 65 * 2 + 2


def tree_algorithmic_bytes(work: dict, n_eval: int, history: int) -> dict:
    """The tree kernels' algorithmic bytes (TREE_BYTES) over a window's
    engine counters (oamd_engine_tree_work): total and per tree launch."""
    b = (TREE_BYTES["per_child_scanned"] * work["children_scanned"] + TREE_BYTES["per_level"] * work["levels"]
         + TREE_BYTES["per_expansion"] * work["expansions"]
         + TREE_BYTES["per_child_created"] * work["children_created"] + tree_bytes_per_row(history) * n_eval)
    return {"bytes": b, "per_launch": b / max(1, work["launches"])}


def resnet_weight_bytes(in_ch: int, C: int, R: int, hidden: int, dtype_bytes: int = 2) -> int:
    """Algorithmic weight bytes of one launch (BN folded): the 3x3 convolutions
    in the compute dtype, biases and heads in fp32."""
    convs = 9 * in_ch * C + 2 * R * 9 * C * C
    small = (1 + 2 * R) * C + (C * 3 + 3) + (128 * 65 + 65) + (64 * hidden + hidden) + (hidden + 1)
    return dtype_bytes * convs + 4 * small


# per evaluated row: packed features in (2 + 2H words of 8 B at H = 8), fp32 policy (65) + value out
RESNET_ROW_BYTES = (2 + 2 * 8) * 8 + 65 * 4 + 4


def resnet_flops_per_eval(in_ch: int, C: int, R: int, hidden: int) -> float:
    conv0 = 2 * 64 * 9 * in_ch * C
    tower = 2 * R * 2 * 64 * 9 * C * C
    heads = 2 * 64 * C * 3 + 2 * 128 * 65 + 2 * 64 * hidden + 2 * hidden
    return float(conv0 + tower + heads)


# ---- CPU baseline (configs[0]) ----------------------------------------------

def usable_cpus() -> dict:
    """CPUs this process may run on: the affinity mask, capped by a cgroup v2
    CPU quota (a GPU box grants a share of a larger machine; os.cpu_count()
    shows the whole machine)."""
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = nproc
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        quota = None
    usable = min(affinity, quota) if quota else affinity
    return {"nproc": nproc, "affinity_cpus": affinity, "cgroup_quota_cpus": quota, "usable": usable}


def cpu_baseline(history: int, C: int, R: int, hidden: int, moves: int = 24, warmup_moves: int = 2,
                 threads: int | None = None, max_seconds: float = 120.0, seed: int = 1) -> dict:
    """Oracle port of the reference CPU path (configs[0]): 1 game from the
    initial position, 2 threads x 16, 800 sims/move, eps 0.25, fp32 torch-CPU
    ResNet; `warmup_moves` untimed moves, then `moves` timed ones (stopping
    early only past `max_seconds`). The game is fixed by its random-stream key,
    so every box times the same positions. torch intra-op threads = `threads`
    (default: every CPU this process may use, BASELINE.md "CPU-baseline
    plan"). Validated against the compiled reference in the build container:
    tools/cpu_baseline_validate.py, profiles/r03_cpu_baseline_validation.json."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import numpy as np

    import oracle as O
    import resnet_ref
    from othello_mcts.synthetic import live_state_dict

    cpus = usable_cpus()
    if threads is None:
        threads = cpus["usable"]
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        sd = {k: torch.from_numpy(np.asarray(v)) for k, v in
              live_state_dict(seed, 1 + 2 * history, C, R, hidden).items()}

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
        done = 0
        t0 = time.perf_counter()
        while done < moves and time.perf_counter() - t0 < max_seconds:
            sims += move()
            done += 1
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev_threads)
    return {"value": round(sims / dt, 1), "unit": "simulations/s", "cores": cpus["usable"], "threads": threads,
            "kind": "port", "cpu_model": cpu_model(), "nproc": cpus["nproc"],
            "affinity_cpus": cpus["affinity_cpus"], "cgroup_quota_cpus": cpus["cgroup_quota_cpus"],
            "moves": done, "warmup_moves": warmup_moves,
            "sample": f"1 game from the initial position, {warmup_moves} warm-up + {done} timed moves x 800 sims "
                      f"(T=2 x B=16, eps=0.25), {C}x{R + 1}b fp32 torch-CPU with {threads} threads "
                      f"(the bench's live net, seed {seed}), {dt:.1f} s"}


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ---- multi-GPU plumbing (one process per GPU; games shard, no data-path
# collective). Device-agnostic, so tests/test_dist_cpu.py runs it with gloo.

def dist_env() -> tuple[int, int, int]:
    """(world, rank, local_rank) from the torchrun environment (1, 0, 0 if unset)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def under_launcher() -> bool:
    return "WORLD_SIZE" in os.environ


def shard_seeds(seed: int, rank: int) -> tuple[int, int]:
    """Per-rank (engine RNG key, opening seed): every rank plays its own games."""
    return seed + 7919 * rank, seed + rank


def grouped() -> bool:
    """True when this rank runs in a process group (every launcher run, world 1
    included: the barrier, the MAX reduction and the rank table then go
    through the job's backend, RCCL on the GPU box)."""
    return dist.is_available() and dist.is_initialized()


def cpu_seconds() -> float:
    """Host CPU seconds (user + system) of this process, every thread."""
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def timed_max(world: int, run, sync, device: str) -> tuple[float, float, float]:
    """Run `run()` bracketed by barrier + device sync on both sides; return the
    MAX wall time over ranks (the whole job's time: barrier to barrier), this
    rank's own time (its start barrier to its own final sync, before it waits
    for the others: a slow rank shows here) and the host CPU seconds this
    rank's process spent over its own time (getrusage)."""
    if grouped():
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    c0 = cpu_seconds()
    run()
    sync()
    own = time.perf_counter() - t0
    cpu = cpu_seconds() - c0
    if grouped():
        dist.barrier()
    job = time.perf_counter() - t0
    t = torch.tensor([job], dtype=torch.float64, device=device)
    if grouped():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), own, cpu


def rank_table(world: int, rank: int, device_id: str, sims: int, own_s: float | None = None,
               cpu_s: float | None = None) -> list[dict]:
    """[{rank, device, sims, ms, sims_per_s, cpu_s_per_s}] of every rank
    (all_gather_object over the job's process group): which physical device
    each rank ran on, its units, its own time (start barrier to its own final
    sync; the line's value uses the MAX over ranks of the barrier-to-barrier
    time, so a slow rank shows here) and the host CPU seconds its process used
    per wall second of that time (the host budget: N ranks need N x this of
    the box's CPUs)."""
    me = {"rank": rank, "device": device_id, "sims": sims}
    if own_s is not None:
        me["ms"] = round(own_s * 1e3, 3)
        me["sims_per_s"] = round(sims / own_s, 1)
        if cpu_s is not None:
            me["cpu_s_per_s"] = round(cpu_s / own_s, 3)
    if not grouped():
        return [me]
    out: list = [None] * world
    dist.all_gather_object(out, me)
    return out


def host_budget(ranks: list[dict]) -> dict:
    """The host CPUs the ranks used over the timed region (rank_table's
    cpu_s_per_s) against the CPUs this process may use (usable_cpus: the
    cgroup quota of a GPU box). At the driver's N = 8 the node's ranks need
    8 x the per-rank figure; `fits_8_ranks` compares that with the quota this
    box grants one process (the 8-GPU node's own quota is not visible here)."""
    per = [r["cpu_s_per_s"] for r in ranks if "cpu_s_per_s" in r]
    cpus = usable_cpus()
    out = {"usable_cpus": cpus["usable"], "cgroup_quota_cpus": cpus["cgroup_quota_cpus"], "ranks": len(ranks)}
    if per:
        out.update({"cpu_s_per_s_max": max(per), "cpu_s_per_s_sum": round(sum(per), 3),
                    "need_at_8_ranks": round(8 * max(per), 2), "fits_8_ranks": bool(8 * max(per) <= cpus["usable"])})
    return out


def aggregate_rate(world: int, games: int, sims_per_search: int, steps: int, dt_max: float) -> float:
    """Whole-job simulations/s: the units all ranks processed / the max time."""
    return world * games * sims_per_search * steps / dt_max


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(nproc: int, argv: list[str], port: int) -> list[str]:
    """The driver's own N>1 launch, for a bare `bench.py --gpus N`."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *argv]


def launch_ranks(args, argv: list[str]) -> int:
    """Bare `bench.py --gpus N` (N > 1, no launcher in the environment): start
    the N rank processes as a torch.distributed.run child and return its exit
    code. Runs before any HIP call of this process (device_count() does not
    initialise the GPU on this image), and never execs: the child is a new
    process. Without the gloo rehearsal the GPUs must be there."""
    backend = os.environ.get("OAMD_BENCH_BACKEND", "nccl")
    if not args.dry_run and backend != "gloo":
        have = torch.cuda.device_count()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {have} "
                  "(OAMD_BENCH_BACKEND=gloo rehearses ranks that share GPUs; its line is labelled a "
                  "rehearsal)", file=sys.stderr)
            return 2
    cmd = launch_command(args.gpus, argv, free_port())
    print(f"bench.py: starting {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def check_ranks(args, world: int, backend: str, ranks: list[dict]) -> None:
    """Refuse a line that would misstate the job: ranks != --gpus, or ranks
    sharing GPUs outside the explicit gloo rehearsal."""
    n_devices = len({r["device"] for r in ranks})
    if n_devices < world and backend != "gloo":
        raise SystemExit(f"bench.py: {world} ranks ran on {n_devices} distinct device(s); every rank needs its "
                         "own GPU (OAMD_BENCH_BACKEND=gloo rehearses shared GPUs)")


def parse_args(argv: list[str]):
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
    ap.add_argument("--nn-chains", type=int, default=2,
                    help="concurrent chains of ResNet launches (1 = every launch serialised)")
    ap.add_argument("--round-robin-endgames", action="store_true",
                    help="all-terminal batches wait for their round instead of the reference's immediate "
                         "re-selection (oamd_engine_set_exact_interleaving(0)); default: exact")
    ap.add_argument("--chain-budget", type=int, default=2,
                    help="re-selections after all-terminal batches per game and round before the chain is split "
                         "(0 = never split; exact interleaving only)")
    ap.add_argument("--chain-cuts", type=int, default=64,
                    help="most chain splits per game and search (= most extra rounds; the engine caps it at "
                         "threads x steps / budget)")
    ap.add_argument("--adaptive-min", type=int, default=1,
                    help="fewest extra rounds of the adaptive count (the margin over the cuts used)")
    ap.add_argument("--fixed-extra-rounds", action="store_true",
                    help="always --chain-cuts extra rounds (no adaptive count)")
    ap.add_argument("--lockstep-moves", action="store_true",
                    help="the multi-move call in lock step (every game waits for the group's slowest at each move, "
                         "chain-splitting extra rounds) instead of free-running games (oamd_engine_set_free_running)")
    ap.add_argument("--extra-grid", type=int, default=128,
                    help="workgroups of the extra rounds' ResNet launches (0 = the regular grid)")
    ap.add_argument("--cpu-baseline-moves", type=int, default=24,
                    help="timed moves of the CPU baseline (0 = skip it), after 2 warm-up moves")
    ap.add_argument("--no-ceiling-probe", dest="ceiling_probe", action="store_false",
                    help="skip the same-box MFMA ceiling probe after the timed regions (roofline.measured_ceiling "
                         "then comes from the committed record)")
    ap.add_argument("--cpu-baseline-threads", type=int, default=0,
                    help="torch threads of the CPU baseline (0 = every CPU this process may use)")
    ap.add_argument("--sustained-moves", type=int, default=64,
                    help="after the timed region, continue the same games this many more moves (endgames, "
                         "restarts) and report them as the line's `sustained` sub-record (0 = skip)")
    ap.add_argument("--seed", type=int, default=2025)
    ap.add_argument("--net", default="live", choices=list(NET_KINDS),
                    help="weights of the headline workload (bench_state_dict)")
    ap.add_argument("--deep-tree-net", default="selfplay", choices=list(NET_KINDS),
                    help="weights of the deep_tree sub-record (default: the self-play trained net)")
    ap.add_argument("--policy-sharpness", type=float, default=1.25,
                    help="the frontier net's prior sharpness (deep_tree; mean largest prior ~0.4)")
    ap.add_argument("--deep-tree-moves", type=int, default=20,
                    help="moves of the deep_tree sub-record from fresh openings (then --sustained-moves more; "
                         "0 = skip it)")
    ap.add_argument("--no-config-records", dest="config_records", action="store_false",
                    help="skip the configs[3] / configs[4]-shard sub-records")
    ap.add_argument("--latency-moves", type=int, default=20,
                    help="moves per setting of the single-game latency sub-record (0 = skip it)")
    ap.add_argument("--sync-search", action="store_true", help="host waits for every search (diagnostic)")
    ap.add_argument("--per-move-calls", action="store_true",
                    help="one search + selfplay_move call pair per step instead of one multi-move call")
    ap.add_argument("--timing-every", type=int, default=5,
                    help="record the kernels' HIP events on every N-th timed search (1 = all; the event "
                         "packets add ~10 us per NN launch boundary to the searches they time)")
    ap.add_argument("--spin-sync", action="store_true",
                    help="end the timed region with a plain torch.cuda.synchronize() (spins a host CPU) instead of a "
                         "blocking-sync event wait first")
    ap.add_argument("--dry-run", action="store_true",
                    help="rank plumbing only: no GPU, no search (gloo, each step a fixed sleep)")
    ap.add_argument("--dry-step-ms", type=float, default=20.0, help="--dry-run: ms per step (rank r: x (1 + r))")
    args = ap.parse_args(argv)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    return args


class DryWorkload:
    """--dry-run: the bench's rank path with a fixed sleep per step instead of
    the GPU search (rank r sleeps (1 + r) x dry_step_ms, so the max over ranks
    is the last rank's)."""

    def __init__(self, args, rank: int, local: int) -> None:
        self.args = args
        self.rank = rank
        self.device_id = f"{socket.gethostname()}:dry{local}"

    def step(self) -> None:
        time.sleep(self.args.dry_step_ms * 1e-3 * (1 + self.rank))

    def sync(self) -> None:
        pass


def main(argv: list[str] | None = None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus > 1 and not under_launcher():
        raise SystemExit(launch_ranks(args, argv))
    world, rank, local = dist_env()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    # OAMD_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share
    # devices round-robin, timing reduced over gloo); the driver's runs use RCCL
    backend = "gloo" if args.dry_run else os.environ.get("OAMD_BENCH_BACKEND", "nccl")
    if args.dry_run:
        if under_launcher():
            dist.init_process_group("gloo")
        return report(args, world, rank, backend, DryWorkload(args, rank, local))
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    elif local >= torch.cuda.device_count():
        raise SystemExit(f"bench.py: rank {rank} (local {local}) has no GPU: "
                         f"{torch.cuda.device_count()} visible")
    torch.cuda.set_device(local)
    # under a launcher the rank joins the job's process group at every world
    # size (torchrun --nproc-per-node 1 runs the RCCL init, barrier, MAX
    # all-reduce and rank table too); a bare world-1 run has none
    if under_launcher():
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return report(args, world, rank, backend, EngineWorkload(args, rank, local))


NET_KINDS = ("live", "frontier", "selfplay", "torch-default")


def bench_state_dict(kind: str, seed: int, in_ch: int, C: int, R: int, hidden: int, sharpness: float = 1.25) -> dict:
    """Seeded synthetic weights of the benched AlphaZeroNet architecture:
    "live" (the headline net: He-scaled convs, BN statistics of real positions,
    a value head spread over [-1, 1], near-uniform priors;
    synthetic.live_state_dict), "frontier" (the same tower with priors peaked
    on plausible moves), "selfplay" (the deep_tree net: 128x10b H=8 trained by
    self-play, bench_nets/; synthetic.selfplay_state_dict) or "torch-default"
    (round 1-4's init: the tower forgets its input, constant value, uniform
    priors — kept for comparison only)."""
    from othello_mcts.synthetic import alphazero_state_dict, live_state_dict, selfplay_state_dict

    if kind == "live":
        return live_state_dict(seed, in_ch, C, R, hidden)
    if kind == "frontier":
        return live_state_dict(seed, in_ch, C, R, hidden, policy="frontier", policy_sharpness=sharpness)
    if kind == "selfplay":
        if (in_ch, C, R, hidden) != (17, 128, 9, 128):
            raise SystemExit("bench.py: the self-play trained net is 128x10b with history 8")
        return selfplay_state_dict()
    if kind == "torch-default":
        return alphazero_state_dict(seed, in_ch, C, R, hidden)
    raise ValueError(kind)


class EngineWorkload:
    """configs[1] on this rank's GPU: `games` self-play games, one step = one
    search of every game + the on-device self-play move."""

    def __init__(self, args, rank: int, local: int, net_kind: str | None = None) -> None:
        import othello_mcts as om
        from othello_mcts import provenance

        # the loaded liboamd.so must be the one built from the sources on disk
        # (tools/gpu.sh benchvar swaps in prebuilt A/B variants and says so)
        if os.environ.get("OAMD_AB_VARIANT"):
            self.source_hashes = {"variant": os.environ["OAMD_AB_VARIANT"]}
        else:
            self.source_hashes = provenance.check_loaded_library()

        self.args = args
        self.local = local
        self.net_kind = net_kind or args.net
        R = args.blocks - 1
        self.sd = bench_state_dict(self.net_kind, args.seed, 1 + 2 * args.history, args.channels, R, args.hidden,
                                   args.policy_sharpness)
        self.net = om.NativeNet(self.sd, device=local, dtype=args.dtype)
        engine_seed, opening_seed = shard_seeds(args.seed, rank)
        self.b = om.BatchedMCTS(args.games, history_size=args.history, num_simulations=args.sims,
                                num_threads=args.threads, batch_size=args.batch, seed=engine_seed)
        self.b.random_openings(8, seed=opening_seed)
        if args.eval_batch:  # rows per ResNet launch; the 2 pipeline groups stay
            self.b.engine.set_nn_batch(args.eval_batch)
        if args.pipeline:
            self.b.engine.set_pipeline(args.pipeline)
        self.b.engine.set_nn_chains(args.nn_chains)
        self.b.engine.set_exact_interleaving(not args.round_robin_endgames)
        self.b.engine.set_chain_split(args.chain_budget, args.chain_cuts)
        self.b.engine.set_extra_round_grid(args.extra_grid)
        self.b.engine.set_adaptive_extra_rounds(not args.fixed_extra_rounds, args.adaptive_min)
        self.b.engine.set_free_running(not args.lockstep_moves)
        props = torch.cuda.get_device_properties(local)
        self.device_id = f"{os.uname().nodename}:{getattr(props, 'uuid', local)}"

    def step(self) -> None:
        self.b.search(self.net, sync=self.args.sync_search)  # enqueue only; the timed region syncs at its end
        self.b.selfplay_move(temperature_moves=12, opening_moves=8, emit_targets=True)

    def steps(self, n: int) -> None:
        """n steps: one multi-move self-play call (oamd_engine_selfplay_steps, the
        same kernels per game as n x step(); each pipeline group's move and next
        selection overlap the other group's ResNet launch), or n x step() with
        --per-move-calls / --sync-search."""
        if self.args.per_move_calls or self.args.sync_search:
            for _ in range(n):
                self.step()
        else:
            self.b.selfplay_steps(self.net, n, temperature_moves=12, opening_moves=8, emit_targets=True,
                                  keep_all=False)

    def sync(self) -> None:
        """torch.cuda.synchronize(), preceded by polling an event of the stream
        the engine joins its pipeline groups into, 100 us sleeps between polls
        (the host thread sleeps instead of spinning a CPU through the timed
        region; the poll adds <= 0.1 ms to it; --spin-sync: the plain
        synchronize)."""
        if not self.args.spin_sync:
            ev = torch.cuda.Event()
            ev.record()
            while not ev.query():
                time.sleep(1e-4)
        torch.cuda.synchronize()

    def start_measuring(self, every: int | None = None) -> None:
        e = self.b.engine
        e.enable_timing(max(1, self.args.timing_every if every is None else every))
        self.t0 = (e.nn_timing(), e.tree_timing(), e.work_counters(), e.nn_busy(), e.round_counts(),
                   e.descent_depths(), e.tree_work())

    def stop_measuring(self) -> dict:
        e = self.b.engine
        (ms0, la0, rw0), (se0, bk0, tl0), (si0, ev0), (bu0, bl0), (sc0, ro0, fl0), (lv0, ds0, _), tw0 = self.t0
        (ms1, la1, rw1), (se1, bk1, tl1), (si1, ev1), (bu1, bl1), (sc1, ro1, fl1), (lv1, ds1, dmax), tw1 = (
            e.nn_timing(), e.tree_timing(), e.work_counters(), e.nn_busy(), e.round_counts(), e.descent_depths(),
            e.tree_work())
        overflow_games, depth_capped = e.status()
        if overflow_games or depth_capped:
            raise SystemExit(f"bench invalid: {overflow_games} game(s) overflowed their node pool, "
                             f"{depth_capped} hit the depth cap")
        return {"nn_ms": ms1 - ms0, "nn_busy_ms": bu1 - bu0, "busy_launches": bl1 - bl0, "nn_launches": la1 - la0,
                "nn_rows": rw1 - rw0, "select_ms": se1 - se0,
                "backup_ms": bk1 - bk0, "tree_launches": tl1 - tl0, "final_launches": fl1 - fl0,
                "searches": sc1 - sc0, "rounds": ro1 - ro0, "sims": si1 - si0, "evals": ev1 - ev0,
                "overflow_games": overflow_games,
                "depth_mean": (ds1 - ds0) / max(1, lv1 - lv0), "depth_max_since_start": dmax,
                "tree_work": dict(zip(("levels", "children_scanned", "expansions", "children_created", "launches"),
                                      (b - a for a, b in zip(tw0, tw1))))}

    def prior_stats(self, n: int = 256) -> dict:
        """The net's outputs on n real positions (the native kernel itself):
        value spread, mean largest prior, prior mass on legal moves."""
        import numpy as np

        import othello_mcts as om
        from othello_mcts.synthetic import calibration_features

        x = calibration_features(n, self.args.history, self.args.seed + 17)
        out = self.net(torch.from_numpy(x).to(f"cuda:{self.local}"))
        p = out["policy"].float().cpu().numpy()
        v = out["value"].float().cpu().numpy()
        legal = np.zeros((n, 65), bool)
        bits = [1 << (63 - s) for s in range(64)]
        for i in range(n):  # planes 1, 2: black / white; plane 0: white to move
            b = sum(bits[s] for s in range(64) if x[i, 1].flat[s] > 0)
            w = sum(bits[s] for s in range(64) if x[i, 2].flat[s] > 0)
            me, opp = (w, b) if x[i, 0, 0, 0] > 0 else (b, w)
            lm = om.get_legal_moves(me, opp)
            legal[i, :64] = [(lm >> (63 - s)) & 1 == 1 for s in range(64)]
            legal[i, 64] = lm == 0
        mass = (p * legal).sum(1)
        share = (p * legal).max(1) / np.maximum(mass, 1e-30)
        return {"positions": n, "value_std": round(float(v.std()), 4), "value_mean": round(float(v.mean()), 4),
                "mean_max_prior": round(float(p.max(1).mean()), 4),
                "mean_legal_mass": round(float(mass.mean()), 4),
                "mean_max_legal_share": round(float(share.mean()), 4),
                "policy_entropy_nats": round(float(-(p * np.log(np.maximum(p, 1e-30))).sum(1).mean()), 3)}


def run_window(args, wl, world: int, backend: str, n: int,
               every: int | None = None) -> tuple[float, float, dict | None, float]:
    """n steps of `wl` in a barrier-bracketed region, the engine's counters
    over it: (max-over-ranks seconds, this rank's seconds, measurements, this
    rank's host CPU seconds)."""
    measuring = hasattr(wl, "start_measuring")
    if measuring:
        wl.start_measuring(every)

    def run():
        if hasattr(wl, "steps"):
            wl.steps(n)
        else:
            for _ in range(n):
                wl.step()

    dt_max, own, cpu = timed_max(world, run, wl.sync, "cuda" if backend == "nccl" else "cpu")
    return dt_max, own, (wl.stop_measuring() if measuring else None), cpu


def park_barrier(group) -> None:
    """Barrier over a gloo group: waiting ranks block in a socket read (no host
    core spins) while rank 0 times the CPU baseline."""
    if group is not None:
        dist.barrier(group=group)


def report(args, world: int, rank: int, backend: str, wl) -> None:
    L = args.threads * args.batch
    sims_per_search = L * ((args.sims + L - 1) // L)
    dev = "cuda" if backend == "nccl" else "cpu"
    # a host-side group for parking ranks without spinning (RCCL's barrier
    # waits on the device); the dry run's default group is gloo already
    park = None
    if grouped():
        park = dist.new_group(backend="gloo") if backend == "nccl" else dist.group.WORLD
    if hasattr(wl, "steps"):
        wl.steps(args.warmup)
    else:
        for _ in range(args.warmup):
            wl.step()
    wl.sync()
    dt_max, own, m, cpu_s = run_window(args, wl, world, backend, args.steps)
    sustained = None
    if m is not None and args.sustained_moves > 0:
        # the engine's real workload: the same games played on through their
        # endgames (all-terminal batches, chain splitting) and restarts (the
        # roofline covers every launch; HIP events sample every 5th search)
        dt_s, _, ms_, _ = run_window(args, wl, world, backend, args.sustained_moves)
        sustained = sustained_fields(args, ms_, world, sims_per_search, dt_s)
    value = aggregate_rate(world, args.games, sims_per_search, args.steps, dt_max)
    ranks = rank_table(world, rank, wl.device_id, args.games * sims_per_search * args.steps, own, cpu_s)
    check_ranks(args, world, backend, ranks)
    n_devices = len({r["device"] for r in ranks})
    workload = (f"{args.games} concurrent self-play games per GPU, {args.sims} sims/move, "
                f"{args.channels}x{args.blocks}b ResNet {args.dtype}, history {args.history}, "
                f"{args.threads} threads x {args.batch} leaves per step"
                + (f", eval batch {args.eval_batch}" if args.eval_batch else "")
                + (" (BASELINE configs[1])" if (args.games, args.channels, args.blocks, args.sims, args.dtype,
                                                args.eval_batch) == (256, 128, 10, 800, "bf16", 0) else ""))
    net_note = {"live": "seeded live-init (He-scaled convs, BN statistics of real positions, value spread over "
                        "[-1, 1]; synthetic.live_state_dict)",
                "frontier": "seeded live-init with priors peaked on frontier squares (synthetic.live_state_dict "
                            "policy='frontier')",
                "selfplay": "self-play trained (bench_nets/selfplay_128x10b_h8)",
                "torch-default": "seeded torch-default init (degenerate: constant value, uniform priors)"}[args.net]
    result = {
        "metric": METRIC,
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
        "data": (f"synthetic: {net_note} {args.channels}x{args.blocks}b AlphaZeroNet weights, "
                 "random openings (0-8 plies)") if m is not None else
                "DRY RUN: rank plumbing only, no GPU work (each step a fixed sleep); not a measurement",
        "config": {
            "workload": workload,
            "games_per_gpu": args.games,
            "sims_per_move": args.sims,
            "leaves_per_step": L,
            "net_init": args.net,
            "parallelism": (f"games sharded over {world} rank(s) on {n_devices} GPU(s), no collective"
                            + (" (REHEARSAL: ranks share GPUs; not a scaling point)"
                               if n_devices < world else "")),
            "ranks": ranks,
            "backend": (backend if grouped() else "none"),
            "endgame_interleaving": ("round-robin" if args.round_robin_endgames else
                                     f"exact (reference), chains split after {args.chain_budget} re-selections, "
                                     f"<= X times per search, X extra rounds, X adaptive in "
                                     f"[{min(args.adaptive_min, args.chain_cuts)}, {args.chain_cuts}]"
                                     if not args.fixed_extra_rounds else
                                     f"<= {args.chain_cuts} times per search"),
            "calls": ("search + selfplay_move per step" if args.per_move_calls or args.sync_search
                      else f"one selfplay_steps call for the {args.steps} timed steps"
                      + (", games in lock step (extra rounds)" if args.lockstep_moves else
                         ", free-running games (each game's move runs in the round its search completes)")),
        },
    }
    if args.dry_run:
        result["dry_run"] = True
    result["host"] = host_budget(ranks)
    if m is not None:
        result.update(measured_fields(args, m, workload))
        result["net_outputs"] = wl.prior_stats()
        if sustained is not None:
            result["sustained"] = sustained
        if args.deep_tree_moves > 0:
            result["deep_tree"] = deep_tree_record(args, wl, world, rank, backend, sims_per_search)
        if args.config_records:
            result["other_configs"] = config_records(args, wl, world, rank, backend)
        if args.latency_moves > 0 and rank == 0:
            result["latency"] = latency_record(args, wl)
    # the MFMA ceiling on this box (rank 0's GPU), after every timed region
    if m is not None and rank == 0 and args.ceiling_probe:
        rl = [(args.dtype, result["roofline"])] + [(v.get("dtype"), v["roofline"])
                                                   for v in result.get("other_configs", {}).values()]
        got = same_box_ceiling({d for d, _ in rl})
        for d, r in rl:
            if d in got:
                with_ceiling(r, got[d], "this box: tools/mfma_ceiling.hip after the timed regions")
    # the CPU baseline on rank 0 at every world size, after every timed region;
    # the other ranks wait at a gloo barrier (blocked, not spinning)
    if args.cpu_baseline_moves > 0 and (m is not None or args.dry_run):
        if rank == 0:
            dry = args.dry_run
            result["cpu_baseline"] = cpu_baseline(args.history, args.channels, args.blocks - 1, args.hidden,
                                                  moves=1 if dry else args.cpu_baseline_moves,
                                                  warmup_moves=0 if dry else 2,
                                                  threads=args.cpu_baseline_threads or None, seed=args.seed)
            if dry:
                result["cpu_baseline"]["note"] = "dry run: 1 move, no warm-up (plumbing only)"
            result["cpu_baseline"]["world_size"] = world
        park_barrier(park)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if grouped():
        dist.destroy_process_group()


def deep_tree_record(args, wl, world: int, rank: int, backend: str, sims_per_search: int) -> dict:
    """the same configs[1] engine with a net whose priors and
    values are a trained one's (default: the self-play trained net, bench_nets/):
    tree shape (descent depth), k_tree time per round against the ResNet's busy
    time per launch, and whether the tree rounds still hide behind the other
    pipeline group's ResNet launches (step time vs the union busy time)."""
    import copy
    import gc

    del wl.b
    gc.collect()
    torch.cuda.synchronize()
    dw = EngineWorkload(args, rank, wl.local, net_kind=args.deep_tree_net)
    dw.steps(args.warmup)
    dw.sync()
    desc = {"selfplay": "128x10b trained by self-play (bench_nets/selfplay_128x10b_h8, tools/selfplay_train.py: "
                        "15k games from a live init)",
            "frontier": f"live init, priors peaked on frontier squares (sharpness {args.policy_sharpness})"}
    out = {"net": desc.get(args.deep_tree_net, args.deep_tree_net), "net_outputs": dw.prior_stats()}
    for name, n in (("from_openings", args.deep_tree_moves), ("sustained", args.sustained_moves)):
        if n <= 0:
            continue
        dt, _, m, _ = run_window(args, dw, world, backend, n, every=1)
        a = copy.copy(args)
        a.steps = n  # the window's own moves (rows launched)
        mf = measured_fields(a, m, "")
        step_ms = dt * 1e3 / n
        busy_per_step = m["nn_busy_ms"] / n
        tree_round_ms = m["select_ms"] / max(1, m["tree_launches"])
        out[name] = {
            "moves": n,
            "value": round(aggregate_rate(world, args.games, sims_per_search, n, dt), 1),
            "unit": "simulations/s",
            "ms_per_step": round(step_ms, 3),
            "depth_mean": round(m["depth_mean"], 3),
            "depth_max": m["depth_max_since_start"],
            "k_tree_ms_per_round": round(tree_round_ms, 4),
            "resnet_busy_ms_per_launch": mf["roofline"]["busy_ms_per_launch"],
            "resnet_busy_union_ms_per_step": round(busy_per_step, 3),
            "step_over_busy": round(step_ms / max(busy_per_step, 1e-9), 4),
            "k_tree_hidden": bool(step_ms <= 1.05 * busy_per_step),
            "rounds_per_search": mf["tree_kernels"]["rounds_per_search"],
            "terminal_share": mf["work"]["terminal_share"],
            "frac": mf["roofline"]["frac"],
        }
    out["note"] = ("timed on every search (HIP events on every round: the event packets lengthen the launch "
                   "gaps ~10 us, so this rate is a little below an untimed run's); depth = levels below the root of "
                   "every selected leaf; k_tree_hidden: step time within 5 % of the union of the ResNet launches' "
                   "busy intervals")
    del dw
    return out


def config_records(args, wl, world: int, rank: int, backend: str) -> dict:
    """VERDICT r4 (What's weak 9): configs[3] (256x20b bf16, 1600 sims/move)
    and the per-GPU shard of configs[4] (512 games, 128x10b fp16, eval batch
    2048) in the driver's own line, on short windows after the headline's (the
    same rank path; every rank runs its shard, so at N GPUs configs[4]'s
    record is N x 512 games). Live seeded nets, like the headline's."""
    import copy
    import gc

    if getattr(wl, "b", None) is not None:
        del wl.b
    gc.collect()
    out = {}
    specs = (("configs3", "256x20b ResNet bf16, 256 games per GPU, 1600 sims/move (BASELINE configs[3])",
              dict(channels=256, blocks=20, hidden=256, sims=1600, dtype="bf16", eval_batch=0, games=256), 2, 10),
             ("configs4_shard", "128x10b ResNet fp16, 512 games per GPU, eval batch 2048, 800 sims/move "
              "(BASELINE configs[4]: 4096 games over 8 GPUs)",
              dict(channels=128, blocks=10, hidden=128, sims=800, dtype="fp16", eval_batch=2048, games=512), 2, 10))
    for name, desc, over, warm, n in specs:
        a = copy.copy(args)
        a.__dict__.update(over)
        a.steps = n
        w = EngineWorkload(a, rank, wl.local, net_kind="live")
        w.steps(warm)
        w.sync()
        dt, own, m, _ = run_window(a, w, world, backend, n)
        L = a.threads * a.batch
        sps = L * ((a.sims + L - 1) // L)
        mf = measured_fields(a, m, "")
        r = mf["roofline"]
        out[name] = {"workload": desc, "steps": n, "warmup": warm,
                     "value": round(aggregate_rate(world, a.games, sps, n, dt), 1), "unit": "simulations/s",
                     "ms_per_step": round(dt * 1e3 / n, 3), "this_rank_ms": round(own * 1e3, 3),
                     "dtype": a.dtype,
                     "roofline": {k: r[k] for k in ("bound", "achieved", "peak", "unit", "frac", "busy_ms_per_launch",
                                                    "rows_per_launch", "n_eval_per_launch", "flops_per_row",
                                                    "timed_region_launches", "executed_TFLOP_s",
                                                    "measured_ceiling")},
                     "work": mf["work"], "tree_kernels": mf["tree_kernels"]}
        del w
        gc.collect()
    return out


def latency_record(args, wl) -> dict:
    """Single-game latency through the drop-in MCTS (reference README.md:25:
    < 30 ms per 800-simulation action; player.py:208-259 evaluation at 3200
    sims, eps 0, README.md:195): median / p90 ms per search + visit_counts
    over `latency_moves` moves of one game (argmax play), the headline net."""
    import othello_mcts as om

    out = {"published": "< 30 ms per 800-simulation action, 1x RTX 4090 + 24-core CPU (README.md:25)"}
    for name, sims, eps in (("selfplay_800", 800, 0.25), ("evaluation_3200", 3200, 0.0)):
        mc = om.MCTS(history_size=args.history, torch_device=f"cuda:{wl.local}", num_simulations=sims, num_threads=2,
                     batch_size=16, dirichlet_epsilon=eps, seed=3)
        mc.search(wl.net)  # warm-up
        mc.reset_position()
        ms = []
        for _ in range(args.latency_moves):
            if mc.position().is_terminal():
                mc.reset_position()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mc.search(wl.net)
            vc = mc.visit_counts()  # the result on the host, as the caller sees it
            ms.append((time.perf_counter() - t0) * 1e3)
            acts = mc.position().legal_actions()
            mc.apply_action(acts[max(range(len(vc)), key=vc.__getitem__)])
        ms.sort()
        out[name] = {"sims": sims, "threads": 2, "batch_size": 16, "dirichlet_epsilon": eps, "moves": len(ms),
                     "median_ms": round(ms[len(ms) // 2], 3), "p90_ms": round(ms[min(len(ms) - 1, int(len(ms) * 0.9))], 3),
                     "min_ms": round(ms[0], 3)}
        del mc
    return out


def sustained_fields(args, m: dict, world: int, sims_per_search: int, dt_max: float) -> dict:
    """The `sustained` sub-record: `sustained_moves` more moves of the same
    games right after the timed region (not part of `value`)."""
    import copy

    n = args.sustained_moves
    a = copy.copy(args)
    a.steps = n  # the record's own moves (rows launched, timed-region launches)
    mf = measured_fields(a, m, "")
    r = mf["roofline"]
    return {
        "moves": n,
        "value": round(aggregate_rate(world, args.games, sims_per_search, n, dt_max), 1),
        "unit": "simulations/s",
        "ms_per_step": round(dt_max * 1e3 / n, 3),
        "work": mf["work"],
        "note": (f"the same {args.games} games per GPU continued for {n} moves after the timed region "
                 "(endgames with the reference's interleaving, restarts from random openings)"),
        "roofline": {k: r[k] for k in ("achieved", "peak", "unit", "frac", "avg_launch_ms", "busy_ms_per_launch",
                                       "rows_per_launch", "n_eval_per_launch", "timed_region_launches")},
        "tree_kernels": mf["tree_kernels"],
    }


def traffic_record(name: str, kind: str, workload: str) -> dict | None:
    """A committed PMC traffic summary (profiles/NAME), if it was measured on
    this workload and on the current sources of the kernel family `kind`."""
    f = ROOT / "profiles" / name
    if not f.exists():
        return None
    try:
        tj = json.loads(f.read_text())
    except (ValueError, OSError):
        return None
    if tj.get("workload") != workload or tj.get("kernel_hash") != kernel_hash(kind):
        return None
    return tj


CEILING_PROBES = {"bf16": "regs_random", "fp16": "f16_regs_random"}


def mfma_ceiling(dtype: str) -> dict | None:
    """The MFMA rate this chip sustains on random operands at the clock it
    holds under load (tools/mfma_ceiling.hip: k_resnet_w8's wave tile, operands
    in registers), to read the spec-peak `frac` against: the committed probe
    record (profiles/mfma_ceiling.json); report() replaces it with this box's
    own probe run after the timed regions (same_box_ceiling)."""
    f = ROOT / "profiles" / "mfma_ceiling.json"
    if dtype not in CEILING_PROBES or not f.exists():
        return None
    try:
        c = json.loads(f.read_text())
        tfs = c["probes"][CEILING_PROBES[dtype]]["TFLOP_s"]
        return {"TFLOP_s": float(tfs), "tag": c.get("tag"), "source": "profiles/mfma_ceiling.json (another box)"}
    except (ValueError, OSError, KeyError, TypeError):
        return None


def same_box_ceiling(dtypes) -> dict:
    """{dtype: TFLOP/s} from tools/_build/mfma_ceiling (built by
    __graft_entry__.build()) run as a child process on this rank's GPU after
    every timed region; {} if the probe is missing or fails (the lines then
    keep the committed record)."""
    exe = ROOT / "tools" / "_build" / "mfma_ceiling"
    names = {CEILING_PROBES[d]: d for d in dtypes if d in CEILING_PROBES}
    if not names or not exe.exists():
        return {}
    try:
        r = subprocess.run([str(exe), ",".join(names)], capture_output=True, text=True, timeout=120)
    except (OSError, subprocess.TimeoutExpired):
        return {}
    out = {}
    for ln in r.stdout.splitlines():
        try:
            j = json.loads(ln)
        except ValueError:
            continue
        if j.get("probe") in names:
            out[names[j["probe"]]] = float(j["TFLOP_s"])
    return out


def with_ceiling(roofline: dict, tfs: float, source: str) -> None:
    """roofline.measured_ceiling = `tfs`, with the achieved (algorithmic) and
    executed rates as fractions of it."""
    c = {"TFLOP_s": round(tfs, 1), "source": source}
    if "achieved" in roofline:
        c["frac_achieved"] = round(roofline["achieved"] / tfs, 4)
    if "executed_TFLOP_s" in roofline:
        c["frac_executed"] = round(roofline["executed_TFLOP_s"] / tfs, 4)
    roofline["measured_ceiling"] = c


def measured_fields(args, m: dict, workload: str) -> dict:
    """roofline (the fused ResNet kernel), tree-kernel timings and the work
    counters of this rank's timed region."""
    R = args.blocks - 1
    flops = resnet_flops_per_eval(1 + 2 * args.history, args.channels, R, args.hidden)
    # the sampled searches' HIP-event span per launch (includes time a launch
    # shared the CUs with the other NN chain's launch)
    avg_ms = m["nn_ms"] / max(1, m["nn_launches"])
    # busy: the union of the kernel-recorded execution intervals of EVERY
    # ResNet launch in the window (oamd_engine_nn_busy), per launch
    busy_ms = m["nn_busy_ms"] / max(1, m["busy_launches"])
    rows_per_launch = m["nn_rows"] / max(1, m["nn_launches"])
    # n_eval: rows of non-terminal leaves (the MFMA fraction is
    # over evaluated simulations); terminal rows are launched but their
    # workgroups stop at the prologue when a whole workgroup is terminal
    rows_launched = args.games * args.threads * args.batch * ((args.sims + args.threads * args.batch - 1)
                                                              // (args.threads * args.batch)) * args.steps
    eval_share = m["evals"] / max(1, rows_launched)
    # the window's NN rows (every search, every round), over the window's
    # launches: rows, launches and busy time cover the same launches
    n_eval_per_launch = m["evals"] / max(1, m["busy_launches"])
    achieved = flops * n_eval_per_launch / (busy_ms * 1e-3) / 1e12
    # every launched row counted as work (the round-2 basis): n_eval / eval_share
    achieved_launched = achieved / max(eval_share, 1e-9)
    executed = flops - 2.0 * 64 * 9 * args.channels * args.channels * 2 * R // 12
    peak = PEAK_TFLOPS[args.dtype]
    # HBM bytes per launch from the committed PMC summary of this same workload
    # AND the same kernel sources (kernel_hash)
    traffic = None
    tj = traffic_record("traffic_resnet.json", "resnet", workload)
    if tj and tj.get("rows_per_launch") == int(rows_per_launch):
        traffic = tj.get("bytes_per_launch")
    # algorithmic bytes of one launch: the weights once + every evaluated row's
    # features in and policy / value out
    alg_nn = (resnet_weight_bytes(1 + 2 * args.history, args.channels, R, args.hidden)
              + RESNET_ROW_BYTES * n_eval_per_launch)
    tree_bytes = {}
    tj = traffic_record("traffic_tree.json", "tree", workload)
    if tj:
        try:
            tree_bytes = {k: v["bytes_per_launch"] for k, v in tj["kernels"].items()}
        except (KeyError, TypeError):
            tree_bytes = {}
    # k_tree: one launch per search round and pipeline group; "select" rounds
    # back up the previous batch and select the next, the final round backs up
    # rounds per search: every selecting round (the chain-splitting extra
    # rounds included; their count adapts per search) + the final backup
    rounds = m["rounds"] / m["searches"] if m.get("searches") else float(max_search_rounds(args))
    tree = {"bound": "latency", "sims_per_launch": int(rows_per_launch), "rounds_per_search": round(rounds, 3),
            "max_rounds_per_search": max_search_rounds(args), "kernel_hash": kernel_hash("tree")}
    alg_tree = tree_algorithmic_bytes(m["tree_work"], m["evals"], args.history) if "tree_work" in m else None
    for name, ms, n in (("k_tree", m["select_ms"], m["tree_launches"]),
                        ("k_tree_final_backup", m["backup_ms"], m["final_launches"])):
        avg = ms / max(1, n)
        entry = {"avg_launch_ms": round(avg, 4)}
        if name == "k_tree" and alg_tree is not None:
            tw = m["tree_work"]
            sims = max(1, m["sims"])
            # every k_tree* launch of the window (select rounds, extra rounds,
            # final backups, free-running rounds): the PMC record averages the same set
            entry.update({"algorithmic_bytes_per_launch": round(alg_tree["per_launch"]),
                          "algorithmic_bytes_per_sim": round(alg_tree["bytes"] / sims, 1),
                          "byte_model": {"constants": TREE_BYTES, "per_nn_row": tree_bytes_per_row(args.history),
                                         "window": tw,
                                         "children_scanned_per_level": round(tw["children_scanned"]
                                                                             / max(1, tw["levels"]), 3),
                                         "children_per_expansion": round(tw["children_created"]
                                                                         / max(1, tw["expansions"]), 3),
                                         "source": "SURVEY.md §8(d) per-item bytes x the engine's counters "
                                                   "(oamd_engine_tree_work) over the timed region"}})
        if name in tree_bytes:
            gbs = tree_bytes[name] / (avg * 1e-3) / 1e9
            entry.update({"hbm_bytes_per_launch": tree_bytes[name], "achieved_GB_s": round(gbs, 2),
                          "frac_hbm_peak": round(gbs / PEAK_HBM_GBS, 5)})
            if "algorithmic_bytes_per_launch" in entry:
                entry["counter_over_algorithmic"] = round(tree_bytes[name] / max(1.0, alg_tree["per_launch"]), 3)
        tree[name] = entry
    executed_tfs = executed * n_eval_per_launch / (busy_ms * 1e-3) / 1e12
    ceiling = mfma_ceiling(args.dtype)
    if ceiling:
        # algorithmic and executed rates against the measured random-data ceiling
        ceiling.update({"frac_achieved": round(achieved / ceiling["TFLOP_s"], 4),
                        "frac_executed": round(executed_tfs / ceiling["TFLOP_s"], 4)})
    return {
        "overflow_games": m["overflow_games"],
        "work": {"simulations": m["sims"], "n_eval": m["evals"], "rows_launched": rows_launched,
                 "terminal_share": round(1.0 - eval_share, 5),
                 # tree shape: levels below the root of every selected leaf
                 "depth_mean": round(m["depth_mean"], 3), "depth_max_since_start": m["depth_max_since_start"]},
        "roofline": {
            "bound": "mfma",
            "kernel": "k_resnet_w8 (fused 19-conv tower + heads, 8-wave geometry)",
            "achieved": round(achieved, 2),
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": round(alg_nn),
            "traffic_over_algorithmic": round(traffic / alg_nn, 2) if traffic else None,
            "basis": ("n_eval rows (non-terminal leaves of every search and round in the timed region) per launch "
                      "x flops_per_row / busy ms per launch (the union of the kernel-recorded execution intervals "
                      "of every ResNet launch in the timed region / those launches)"),
            "launches": m["busy_launches"],
            "timed_region_launches": m["busy_launches"],
            "kernel_hash": kernel_hash("resnet"),
            "library_source_hash": kernel_hash("all"),
            "avg_launch_ms": round(avg_ms, 4),
            "busy_ms_per_launch": round(busy_ms, 4),
            "nn_chains": args.nn_chains,
            "rows_per_launch": int(rows_per_launch),
            "n_eval_per_launch": round(n_eval_per_launch, 1),
            "flops_per_row": flops,
            # every launched row counted as work (the round-2 basis)
            "achieved_rows_launched": round(achieved_launched, 2),
            "frac_rows_launched": round(achieved_launched / peak, 4),
            # the default build leaves out the tower MFMAs whose activations are
            # all zero border (1/12 of every tower conv): achieved
            # counts the algorithmic FLOPs above, these are the ones executed
            "executed_flops_per_row": executed,
            "executed_TFLOP_s": round(executed_tfs, 2),
            "measured_ceiling": ceiling,
        },
        "tree_kernels": tree,
    }


if __name__ == "__main__":
    main()

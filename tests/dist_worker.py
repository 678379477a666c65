"""Worker for tests/test_dist_cpu.py, launched by torch.distributed.run with the
gloo backend on CPU: exercises bench.py's multi-process plumbing (torchrun env
parsing, per-rank game shards, barrier + max-over-ranks timing, whole-job
aggregation) the way the driver's N>1 bench run uses it over RCCL.

Each rank plays its own shard of games with the oracle (the test's checker;
the GPU engine needs a GPU) and rank 0 prints one JSON line."""

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main() -> None:
    world, rank, local = bench.dist_env()
    dist.init_process_group("gloo")
    engine_seed, opening_seed = bench.shard_seeds(2025, rank)
    import oracle as O

    games = 2
    sims = 32
    played = []

    def run():
        # rank r's shard: `games` games with its own keys; rank 1 is slower on purpose
        for g in range(games):
            m = O.OracleMCTS(history_size=2, num_simulations=sims, num_threads=1, batch_size=8,
                             dirichlet_epsilon=0.25, game_key=engine_seed * 16 + g)
            m.search(O.uniform_stub)
            played.append(m.visit_counts())
        time.sleep(0.2 * rank)

    dt_max = bench.timed_max(world, run, lambda: None, "cpu")
    rate = bench.aggregate_rate(world, games, sims, 1, dt_max)
    shards = [None] * world
    dist.all_gather_object(shards, {"rank": rank, "local": local, "seeds": [engine_seed, opening_seed],
                                    "dt_max": dt_max, "played": played})
    # which device each rank ran on (here: one CPU "device" per local rank)
    ranks = bench.rank_table(world, rank, f"cpu{local}", games * sims)
    if rank == 0:
        print(json.dumps({"world": world, "rate": rate, "dt_max": dt_max, "shards": shards,
                          "ranks": ranks}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

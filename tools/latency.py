"""Single-game latency per action (reference README.md:25
"< 30 ms per action, 800 sims" on 1x RTX 4090): the drop-in ``MCTS`` class on
one game with the fused native ResNet, as ``player.py``/``train.py`` use it.

Prints one JSON line per setting: median / p90 ms per ``search`` over the
moves of one game (argmax play), for self-play settings (800 sims, T=2 x B=16,
eps=0.25) and evaluation settings (3200 sims, eps=0, README.md:195).
Seeded live 128x10b weights (the bench's). LAT_DTYPE=fp16 (default bf16):
the NativeNet the drop-in MCTS converts a module to since round 6."""

import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))

import torch  # noqa: E402

import othello_mcts as om  # noqa: E402
from othello_mcts.synthetic import live_state_dict  # noqa: E402


def run(net, sims, eps, moves):
    m = om.MCTS(history_size=8, torch_device="cuda:0", num_simulations=sims, num_threads=2, batch_size=16,
                dirichlet_epsilon=eps, seed=3)
    m.search(net)  # warm-up
    m.reset_position()
    ms = []
    for _ in range(moves):
        if m.position().is_terminal():
            m.reset_position()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.search(net)
        vc = m.visit_counts()  # results on the host, as the caller sees them
        ms.append((time.perf_counter() - t0) * 1e3)
        actions = m.position().legal_actions()
        m.apply_action(actions[max(range(len(vc)), key=vc.__getitem__)])
    ms.sort()
    return {"setting": f"{sims} sims, T=2 x B=16, eps={eps}", "moves": moves,
            "median_ms": round(ms[len(ms) // 2], 2), "p90_ms": round(ms[int(len(ms) * 0.9)], 2),
            "min_ms": round(ms[0], 2)}


def breakdown(net, sims, moves, eps=0.25):
    """Kernel time per move of the same single-game search (HIP events): tree
    kernel launches and ResNet launches (with T > 1 threads one game runs them
    thread by thread, a thread's ResNet rows overlapping the next thread's tree
    work, so tree + NN can exceed the wall time)."""
    b = om.BatchedMCTS(1, history_size=8, num_simulations=sims, num_threads=2, batch_size=16, seed=5,
                       dirichlet_epsilon=eps)
    b.search(net)
    b.selfplay_move(temperature_moves=0)
    b.engine.enable_timing(True)
    nn0, l0, _ = b.engine.nn_timing()
    s0, k0, t0_ = b.engine.tree_timing()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(moves):
        b.search(net)
        b.selfplay_move(temperature_moves=0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    nn1, l1, _ = b.engine.nn_timing()
    s1, k1, t1_ = b.engine.tree_timing()
    return {"setting": f"BatchedMCTS(1), {sims} sims, eps={eps}", "moves": moves,
            "wall_ms_per_move": round(wall / moves, 2),
            "tree_launches_per_move": (t1_ - t0_) / moves, "nn_launches_per_move": (l1 - l0) / moves,
            "tree_ms_per_move": round((s1 - s0 + k1 - k0) / moves, 2), "nn_ms_per_move": round((nn1 - nn0) / moves, 2),
            "tree_us_per_launch": round((s1 - s0) / max(1, t1_ - t0_) * 1e3, 1),
            "nn_us_per_launch": round((nn1 - nn0) / max(1, l1 - l0) * 1e3, 1)}


def main():
    net = om.NativeNet(live_state_dict(2025, 17, 128, 9, 128), device=0, dtype=os.environ.get("LAT_DTYPE", "bf16"))
    print(json.dumps({"dtype": net.dtype}), flush=True)
    for sims, eps, moves in ((800, 0.25, 40), (3200, 0.0, 20)):
        print(json.dumps(run(net, sims, eps, moves)), flush=True)
    print(json.dumps(breakdown(net, 800, 20)), flush=True)
    print(json.dumps(breakdown(net, 800, 20, eps=0.0)), flush=True)


if __name__ == "__main__":
    main()

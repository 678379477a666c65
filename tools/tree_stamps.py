"""Diagnostic: where k_tree's time goes over whole games, from the phase
cycle sums of an OAMD_TREE_STAMPS build (tools/gpu.sh `stamps NAME ts` with
abv/ts/liboamd.so built by tools/tree_stamps_build.sh). Plays the bench's
configs[1] games (256 games, 128x10b bf16, T=2 x B=16, 800 sims, random
openings of 0-8 plies) MOVES moves, one search + self-play move at a time, and
prints per move: the wall time, the terminal-leaf share, and k_tree's phases
in cycles (s_memtime): per wave (a game's round), per descent level, per
leaf's post-descent work (virtual loss, path, features) and per backed-up
leaf, plus the longest wave of the move's rounds.
Env: MOVES (default 64), GAMES (256), PIPE (pipeline groups; 1 = no
co-resident ResNet launch of the other group: k_tree's uncontended speed),
BUDGET / CUTS (chain splitting), NET=torch-default (default: the live net)."""
import ctypes
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import othello_mcts as om  # noqa: E402
from othello_mcts.synthetic import alphazero_state_dict, live_state_dict  # noqa: E402

NAMES = ["waves", "cycles", "descent", "levels", "leaves", "post", "backup", "backed_up", "terminal",
         "max_cycles", "batches", "select", "expand", "path_w", "noise", "refill"]
moves = int(os.environ.get("MOVES", "64"))
games = int(os.environ.get("GAMES", "256"))
lib = ctypes.CDLL(str(ROOT / "othello-alphazero_amd" / "othello_mcts" / "liboamd.so"))
buf = (ctypes.c_uint64 * len(NAMES))()


def read(reset=1):
    assert lib.oamd_debug_tree_stamps(buf, ctypes.c_int64(len(NAMES)), ctypes.c_int32(reset)) == 0, \
        "build with -DOAMD_TREE_STAMPS"
    return dict(zip(NAMES, np.frombuffer(buf, dtype=np.uint64).astype(np.int64).tolist()))


net = om.NativeNet(alphazero_state_dict(2025, 17, 128, 9, 128) if os.environ.get("NET") == "torch-default"
                   else live_state_dict(2025, 17, 128, 9, 128), device=0)
b = om.BatchedMCTS(games, history_size=8, num_simulations=int(os.environ.get("SIMS", "800")), num_threads=2,
                   batch_size=16, seed=2025, dirichlet_epsilon=float(os.environ.get("EPS", "0.25")))
b.random_openings(8, seed=2025)
if os.environ.get("PIPE"):
    b.engine.set_pipeline(int(os.environ["PIPE"]))
if os.environ.get("BUDGET"):
    b.engine.set_chain_split(int(os.environ["BUDGET"]), int(os.environ.get("CUTS", "3")))
for _ in range(2):  # warm-up
    b.search(net)
    b.selfplay_move(temperature_moves=12, opening_moves=8)
torch.cuda.synchronize()
read()
tot = {k: 0 for k in NAMES}
print("move  ms    term   waves  cyc/wave  cyc/level  lvl/leaf  post/leaf  bkup/leaf  max_wave_cyc  batches/wave")
for mv in range(moves):
    t0 = time.perf_counter()
    sims, evals = b.search(net)
    b.selfplay_move(temperature_moves=12, opening_moves=8)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    s = read()
    for k in NAMES:
        tot[k] = max(tot[k], s[k]) if k == "max_cycles" else tot[k] + s[k]
    w, lv, lf, bu = max(1, s["waves"]), max(1, s["levels"]), max(1, s["leaves"]), max(1, s["backed_up"])
    print(f"{mv:4d} {ms:6.1f} {1 - evals / sims:6.3f} {s['waves']:6d} {s['cycles'] / w:9.0f} "
          f"{s['descent'] / lv:9.0f} {s['levels'] / lf:8.2f} {s['post'] / lf:9.0f} {s['backup'] / bu:9.0f} "
          f"{s['max_cycles']:12d} {s['batches'] / w:8.2f}", flush=True)
w, lv, lf, bu = max(1, tot["waves"]), max(1, tot["levels"]), max(1, tot["leaves"]), max(1, tot["backed_up"])
print(f"all: cycles/wave {tot['cycles'] / w:.0f}  descent {tot['descent'] / tot['cycles']:.3f}  "
      f"post {tot['post'] / tot['cycles']:.3f}  backup {tot['backup'] / tot['cycles']:.3f} of wave cycles; "
      f"cycles/level {tot['descent'] / lv:.0f}, levels/leaf {tot['levels'] / lf:.2f}, post/leaf "
      f"{tot['post'] / lf:.0f}, backup/leaf {tot['backup'] / bu:.0f} (expansion {tot['expand'] / bu:.0f}, path "
      f"statistics {tot['path_w'] / bu:.0f}), root noise/leaf {tot['noise'] / lf:.0f} (refills {tot['refill'] / lf:.0f}), terminal leaves {tot['terminal'] / lf:.3f}, "
      f"longest wave {tot['max_cycles']}")

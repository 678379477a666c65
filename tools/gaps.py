"""Diagnostic for kernel-trace runs: the bench's self-play loop (256 games,
128x10b) for a few moves with HIP-event timing on/off (TIMING) and a chosen
number of pipeline groups (PIPE), so rocprofv3 --kernel-trace shows the gaps
between consecutive k_resnet launches. Analyse with tools/kt_gaps.py."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))
import torch  # noqa: E402

import othello_mcts as om  # noqa: E402
from othello_mcts.synthetic import alphazero_state_dict  # noqa: E402

net = om.NativeNet(alphazero_state_dict(2025, 17, 128, 9, 128), device=0)
b = om.BatchedMCTS(256, history_size=8, num_simulations=800, num_threads=2, batch_size=16, seed=1)
b.random_openings(8, seed=2)
b.engine.set_pipeline(int(os.environ.get("PIPE", "0")))
b.engine.enable_timing(os.environ.get("TIMING", "0") == "1")
for _ in range(int(os.environ.get("MOVES", "3"))):
    b.search(net, sync=False)
    b.selfplay_move(temperature_moves=12, opening_moves=8, emit_targets=True)
torch.cuda.synchronize()
print("done", flush=True)

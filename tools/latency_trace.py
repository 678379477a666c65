"""Diagnostic: a few single-game searches (the drop-in MCTS; SIMS argv[1],
default 3200, and EPS env, default 0)
for a kernel trace (tools/gpu.sh trace-style: rocprofv3 --kernel-trace --stats
-- python3 tools/latency_trace.py). Prints the per-search wall times."""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))

import torch  # noqa: E402

import othello_mcts as om  # noqa: E402
from othello_mcts.synthetic import live_state_dict  # noqa: E402

sims = int(sys.argv[1]) if len(sys.argv) > 1 else 3200
net = om.NativeNet(live_state_dict(2025, 17, 128, 9, 128), device=0)
m = om.MCTS(history_size=8, torch_device="cuda:0", num_simulations=sims, num_threads=2, batch_size=16,
            dirichlet_epsilon=float(os.environ.get("EPS", "0")), seed=3)
for i in range(8):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.search(net)
    vc = m.visit_counts()
    print(f"search {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
    acts = m.position().legal_actions()
    m.apply_action(acts[max(range(len(vc)), key=vc.__getitem__)])

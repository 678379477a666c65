"""Diagnostic: split k_resnet time into a per-workgroup fixed part and a per-conv
part by timing nets of 1+2R convs (R = 0, 1, 3, 9) at the same row count:
t(R) = fixed + (1 + 2R) x per_conv (least squares). Prints one line per R and the fit."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import othello_mcts as om  # noqa: E402
from othello_mcts.synthetic import alphazero_state_dict  # noqa: E402

rows = 8192
x = (torch.rand((rows, 17, 8, 8), device="cuda") < 0.3).float()
Rs, ts = [], []
for R in (0, 1, 3, 9):
    net = om.NativeNet(alphazero_state_dict(1, 17, 128, R, 128), device=0)
    for _ in range(3):
        net(x)
    torch.cuda.synchronize()
    ms = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            net(x)
        b.record()
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b) / 10)
    t = sorted(ms)[2]
    Rs.append(1 + 2 * R)
    ts.append(t)
    print(f"R={R} convs={1 + 2 * R}: {t:.4f} ms/launch ({rows} rows)", flush=True)
# regress on tower convs (2R); the first conv has 10 of a tower conv's 36 K-steps
A = np.vstack([np.ones(len(Rs)), np.array(Rs, dtype=float) - 1]).T
(f1, per), *_ = np.linalg.lstsq(A, np.array(ts), rcond=None)
fixed = f1 - per * 10 / 36
print(f"fit: {per:.4f} ms per tower conv; first conv + fixed {f1:.4f} ms; fixed (prologue, heads, "
      f"launch, tail) ~{fixed:.4f} ms = {fixed / ts[-1]:.2%} of the R=9 launch")

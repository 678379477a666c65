"""Train a 128x10b net by self-play on one MI355X, the reference's loop in
miniature (train.py:386-521: self-play games -> 8-fold samples with outcome
values -> SGD epochs; README.md:69-90 hyper-parameters: lr 0.02, momentum 0.9,
L2 1e-4, training batch 256, 800 sims, T=2 x B=16, eps 0.25, alpha 0.5,
temperature for the first 12 moves), with this package's pieces: the
on-device self-play driver (BatchedMCTS.selfplay_steps), the HBM sample buffer
(SampleBuffer), the reference loss (alphazero_loss / train_epoch) and the
native net refreshed after every epoch (refresh_native).

Purpose: a benchmark workload whose priors and values are coherent the way a
trained net's are (trees of a trained net concentrate and
descend deeper than those of any random init). Output: the trained state_dict
as float16 (npz, the reference's keys) + a JSON log of the iterations.

Usage (GPU box): python tools/selfplay_train.py OUT_PREFIX [iterations] [games]
"""

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import othello_mcts as om  # noqa: E402
from othello_mcts.synthetic import live_state_dict  # noqa: E402


class AZNet(torch.nn.Module):
    """AlphaZeroNet's layers and state_dict keys (neural_net.py:9-172), for
    training here: the reference module itself does not travel to the box."""

    def __init__(self, in_ch=17, C=128, R=9, hid=128):
        super().__init__()
        nn = torch.nn

        def cb():
            m = nn.Module()
            m.conv = nn.Conv2d(in_ch, C, 3, padding=1)
            m.norm = nn.BatchNorm2d(C)
            return m

        def rb():
            m = nn.Module()
            m.conv1, m.norm1 = nn.Conv2d(C, C, 3, padding=1), nn.BatchNorm2d(C)
            m.conv2, m.norm2 = nn.Conv2d(C, C, 3, padding=1), nn.BatchNorm2d(C)
            return m

        self.conv_block = cb()
        self.residual_blocks = nn.ModuleList([rb() for _ in range(R)])
        ph = nn.Module()
        ph.conv, ph.norm, ph.linear = nn.Conv2d(C, 2, 1), nn.BatchNorm2d(2), nn.Linear(128, 65)
        vh = nn.Module()
        vh.conv, vh.norm = nn.Conv2d(C, 1, 1), nn.BatchNorm2d(1)
        vh.linear1, vh.linear2 = nn.Linear(64, hid), nn.Linear(hid, 1)
        self.policy_head, self.value_head = ph, vh

    def forward(self, x):
        h = F.relu(self.conv_block.norm(self.conv_block.conv(x)))
        for b in self.residual_blocks:
            y = F.relu(b.norm1(b.conv1(h)))
            h = F.relu(b.norm2(b.conv2(y)) + h)
        p = F.relu(self.policy_head.norm(self.policy_head.conv(h)))
        p = torch.softmax(self.policy_head.linear(p.flatten(1)), dim=1)
        v = F.relu(self.value_head.norm(self.value_head.conv(h)))
        v = F.relu(self.value_head.linear1(v.flatten(1)))
        v = torch.tanh(self.value_head.linear2(v).squeeze(1))
        return {"policy": p, "value": v}


def main():
    out = Path(sys.argv[1])
    iterations = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    G = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    moves_per_iter = 64
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    sd0 = live_state_dict(2025, 17, 128, 9, 128)
    model = AZNet().to(dev)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd0.items()})
    native = om.NativeNet(sd0, device=0)
    opt = torch.optim.SGD(model.parameters(), lr=0.02, momentum=0.9)
    b = om.BatchedMCTS(G, history_size=8, num_simulations=800, num_threads=2, batch_size=16,
                       dirichlet_epsilon=0.25, dirichlet_alpha=0.5, seed=77)
    b.reset()
    buf = om.SampleBuffer(G, 17, capacity=400_000, device=dev)
    log = []
    t_start = time.time()
    gen = torch.Generator().manual_seed(1)
    for it in range(iterations):
        t0 = time.time()
        games0 = buf.games_completed
        for _ in range(moves_per_iter // 16):  # 16 moves per call: bounded output buffers
            o = b.selfplay_steps(native, 16, temperature_moves=12, opening_moves=0, emit_targets=True,
                                 keep_all=True)
            for i in range(16):
                buf.add({k: v[i] for k, v in o.items()})
        torch.cuda.synchronize()
        t1 = time.time()
        n = buf.size
        losses = om.train_epoch(model, opt, buf.features[:n], buf.policies[:n], buf.values[:n], 256,
                                l2_weight=1e-4, generator=gen)
        model.eval()
        om.refresh_native(native, model)
        torch.cuda.synchronize()
        rec = {"iteration": it, "games": buf.games_completed, "new_games": buf.games_completed - games0,
               "samples": n, "selfplay_s": round(t1 - t0, 2), "train_s": round(time.time() - t1, 2),
               **{k: round(v, 4) for k, v in losses.items()}}
        log.append(rec)
        print(json.dumps(rec), flush=True)
        if time.time() - t_start > (float(sys.argv[4]) if len(sys.argv) > 4 else 900.0):
            break
    sd = {k: v.detach().float().cpu().numpy() for k, v in model.state_dict().items()}
    np.savez_compressed(str(out) + ".npz", **{k: (v.astype(np.float16) if v.dtype == np.float32 else v)
                                             for k, v in sd.items()})
    Path(str(out) + ".json").write_text(json.dumps({"iterations": log, "games_per_engine": G,
                                                    "moves_per_iteration": moves_per_iter}, indent=1))


if __name__ == "__main__":
    main()

"""Generate the training-loss fixture from the REFERENCE's own ``_train``
(python/othello_alphazero/train.py:455-521), in the build container only.

A tiny AlphaZeroNet (reference class, seeded synthetic weights) takes one SGD
step of ``_train`` over 16 samples (batch 16, so the shuffle does not change
the batch). Recorded: the samples, the parameter values before the step, the
forward outputs the loss saw (train-mode BatchNorm, captured by wrapping the
module's forward), the mean losses ``_train`` returned, and the parameters
after the step. tests/test_cpu_training.py checks
``othello_mcts.training.alphazero_loss`` against it.

Usage: python tests/golden/make_ref_train.py  ->  tests/golden/ref_train.npz, ref_train.json
"""

from __future__ import annotations

import json
import sys
import types
from argparse import Namespace
from pathlib import Path

sys.dont_write_bytecode = True

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
GOLD = ROOT / "tests" / "golden"
sys.path.insert(0, "/root/reference/python")
sys.path.insert(0, str(ROOT / "othello-alphazero_amd" / "othello_mcts"))

pkg = types.ModuleType("othello_mcts")  # train.py imports MCTS at module level; unused here
pkg.MCTS = object
sys.modules["othello_mcts"] = pkg
from othello_alphazero import train  # noqa: E402  reference, read-only
from othello_alphazero.neural_net import AlphaZeroNet  # noqa: E402

from synthetic import alphazero_state_dict, net_config_from_state_dict  # noqa: E402  (this repo)


def main() -> None:
    torch.manual_seed(0)
    torch.set_num_threads(1)
    sd = alphazero_state_dict(31, 9, 16, 2, 16)
    net = AlphaZeroNet(**net_config_from_state_dict(sd))
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    names = [n for n, _ in net.named_parameters()]
    before = {n: p.detach().clone() for n, p in net.named_parameters()}

    rng = np.random.default_rng(5)
    n = 16
    feats = (rng.random((n, 9, 8, 8)) < 0.3).astype(np.float32)
    feats[:, 0] = (rng.random((n, 1, 1)) < 0.5)
    pol = rng.random((n, 65)).astype(np.float32)
    pol /= pol.sum(1, keepdims=True)
    val = rng.choice([-1.0, 0.0, 1.0], size=n).astype(np.float32)
    ds = train._AlphaZeroDataset()
    ds.features = list(torch.from_numpy(feats))
    ds.policies = list(torch.from_numpy(pol))
    ds.values = list(torch.from_numpy(val))

    seen = {}
    orig_forward = net.forward

    def forward(x):
        out = orig_forward(x)
        seen["order"] = x.detach().clone()
        seen["policy"] = out["policy"].detach().clone()
        seen["value"] = out["value"].detach().clone()
        return out

    net.forward = forward
    opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9)
    args = Namespace(training_batch_size=n, training_dataloader_workers=0, pin_memory=False, device="cpu",
                     l2_weight_regulation=1e-4)
    means = train._train(net, opt, ds, args)
    # the batch order the DataLoader chose: map each recorded row back to a sample
    order = [int(np.nonzero((feats == r.numpy()).all(axis=(1, 2, 3)))[0][0]) for r in seen["order"]]
    arrays = {"features": feats, "policy": pol, "value": val, "order": np.array(order, np.int32),
              "out_policy": seen["policy"].numpy(), "out_value": seen["value"].numpy()}
    for k in names:
        arrays["before__" + k] = before[k].numpy()
        arrays["after__" + k] = dict(net.named_parameters())[k].detach().numpy()
    np.savez_compressed(GOLD / "ref_train.npz", **arrays)
    (GOLD / "ref_train.json").write_text(json.dumps({
        "provenance": "reference train._train (train.py:455-521), one SGD step, tests/golden/make_ref_train.py",
        "net": net_config_from_state_dict(sd), "l2_weight": 1e-4, "lr": 0.1, "momentum": 0.9,
        "parameters": names, "mean_losses": means}, indent=1))
    print("losses", means)


if __name__ == "__main__":
    main()

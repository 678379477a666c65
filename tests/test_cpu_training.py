"""Training step beside the engine (othello_mcts/training.py).

The loss is pinned by the REFERENCE's own ``_train`` (train.py:455-521):
tests/golden/make_ref_train.py ran one SGD step of it on a tiny AlphaZeroNet
and recorded the forward outputs the loss saw, the parameters and the losses
it returned. The loop and the device sample buffer are checked for their
semantics (drop_last batches, running means, value targets = SelfPlayCollector's)."""

import json

import numpy as np
import pytest
import torch

from othello_mcts.selfplay import FIN_BLACK, FIN_NONE, FIN_WHITE, SelfPlayCollector
from othello_mcts.training import SampleBuffer, alphazero_loss, train_epoch


@pytest.fixture(scope="module")
def ref(golden_dir):
    meta = json.loads((golden_dir / "ref_train.json").read_text())
    return meta, dict(np.load(golden_dir / "ref_train.npz"))


def test_loss_matches_reference_train(ref):
    meta, a = ref
    order = a["order"]
    params = [torch.from_numpy(a["before__" + k]) for k in meta["parameters"]]
    got = alphazero_loss(torch.from_numpy(a["out_policy"]), torch.from_numpy(a["out_value"]),
                         torch.from_numpy(a["policy"][order]), torch.from_numpy(a["value"][order]),
                         params, meta["l2_weight"])
    for k, v in meta["mean_losses"].items():
        assert got[k].item() == pytest.approx(v, rel=1e-6, abs=0), k


class _Toy(torch.nn.Module):
    def __init__(self, c):
        super().__init__()
        self.lin = torch.nn.Linear(c * 64, 66)

    def forward(self, x):
        y = self.lin(x.flatten(1))
        return {"policy": torch.softmax(y[:, :65], 1), "value": torch.tanh(y[:, 65])}


def test_train_epoch_semantics():
    torch.manual_seed(0)
    n, c = 37, 5
    f = (torch.rand(n, c, 8, 8) < 0.3).float()
    p = torch.softmax(torch.randn(n, 65), 1)
    v = torch.randint(-1, 2, (n,)).float()
    m = _Toy(c)
    m0 = _Toy(c)
    m0.load_state_dict(m.state_dict())
    opt = torch.optim.SGD(m.parameters(), lr=0.0)  # lr 0: every batch sees the same weights
    g = torch.Generator().manual_seed(3)
    means = train_epoch(m, opt, f, p, v, batch_size=8, l2_weight=1e-4, generator=g)
    assert set(means) == {"total_loss", "policy_loss", "value_loss", "l2_loss"}
    # drop_last: 4 full batches of 8; the running means are over those batches
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(3))
    exp = {k: 0.0 for k in means}
    for b in range(4):
        idx = perm[b * 8:(b + 1) * 8]
        out = m0(f[idx])
        ls = alphazero_loss(out["policy"], out["value"], p[idx], v[idx], m0.parameters(), 1e-4)
        for k in exp:
            exp[k] += ls[k].item() / 4
    for k in exp:
        assert means[k] == pytest.approx(exp[k], rel=1e-5)
    assert m.training


def _move(G, C, black_to_move, actions, finished, tag):
    f = torch.zeros((G, 8, C, 8, 8))
    pol = torch.zeros((G, 8, 65))
    for g in range(G):
        f[g, :, 0] = 0.0 if black_to_move[g] else 1.0
        f[g, :, 1, 0, 0] = tag
        pol[g, :, 0] = tag
    return {"actions": torch.tensor(actions, dtype=torch.int32),
            "finished": torch.tensor(finished, dtype=torch.int32), "features": f, "policy": pol}


def test_sample_buffer_matches_collector():
    moves = [
        _move(2, 5, [True, True], [19, 26], [FIN_NONE, FIN_NONE], 1.0),
        _move(2, 5, [False, False], [18, 20], [FIN_NONE, FIN_NONE], 2.0),
        _move(2, 5, [True, False], [64, 21], [FIN_NONE, FIN_WHITE], 3.0),
        _move(2, 5, [False, True], [40, 22], [FIN_BLACK, FIN_NONE], 4.0),
    ]
    col = SelfPlayCollector(2)
    buf = SampleBuffer(2, 5, capacity=64, device="cpu")
    ref = {"features": [], "policies": [], "values": []}
    for mv in moves:
        got = col.add(mv)
        for k in ref:
            ref[k] += got[k]
        buf.add(mv)
    assert buf.size == len(ref["values"]) == 8 * (3 + 4) and buf.games_completed == 2
    # same samples (the buffer stores finished games in completion order)
    torch.testing.assert_close(buf.features[:buf.size], torch.stack(ref["features"]), rtol=0, atol=0)
    torch.testing.assert_close(buf.policies[:buf.size], torch.stack(ref["policies"]), rtol=0, atol=0)
    torch.testing.assert_close(buf.values[:buf.size], torch.stack(ref["values"]), rtol=0, atol=0)
    with pytest.raises(ValueError):
        buf.add({"actions": moves[0]["actions"], "finished": moves[0]["finished"]})

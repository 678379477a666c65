"""Training step beside the native self-play engine.

The reference trains in PyTorch (``_train``, python/othello_alphazero/train.py:
455-521) and so does this package: the optimiser step is plain PyTorch-ROCm on
the user's ``AlphaZeroNet``. What changes is the data path. The reference
moves every self-play sample to the host (``self_play_data()`` returns CPU
tensors, train.py:432-434) and back to the device per minibatch
(train.py:487-489). Here the samples stay in HBM:

* ``SampleBuffer`` appends ``BatchedMCTS.selfplay_move(emit_targets=True)``
  outputs on the device, in the engine's own layout (G, 8, 1+2H, 8, 8) /
  (G, 8, 65), and assigns the value targets of finished games on the device
  (the rule of train.py:438-450, as ``SelfPlayCollector`` does on the host);
* ``train_epoch`` is ``_train``'s loop: shuffled minibatches, ``drop_last``,
  the same loss (``alphazero_loss``, train.py:494-499) and the same returned
  dict of running mean losses (train.py:513-518);
* ``refresh_native`` pushes the updated weights into the ``NativeNet`` the
  engine searches with (one 5.4 MB upload for 128x10b).
"""

from __future__ import annotations

import torch

from .selfplay import FIN_NO_TARGETS, FIN_OVERFLOW, FIN_NONE

_OUTCOME = torch.tensor([0.0, 0.0, 1.0, -1.0])  # finished code (bits 0-1) -> outcome for black


def alphazero_loss(policy: torch.Tensor, value: torch.Tensor, target_policy: torch.Tensor,
                   target_value: torch.Tensor, parameters, l2_weight: float) -> dict[str, torch.Tensor]:
    """train.py:494-499: cross-entropy of the target policy against the net's
    probabilities (not logits), MSE on the value, and an explicit L2 term
    ``l2_weight * sum(p^2)`` over all parameters; total = their sum."""
    policy_loss = -(target_policy * policy.log()).sum(dim=1).mean()
    value_loss = torch.nn.functional.mse_loss(value, target_value)
    l2_loss = l2_weight * sum(p.square().sum() for p in parameters)
    return {"total_loss": policy_loss + value_loss + l2_loss, "policy_loss": policy_loss,
            "value_loss": value_loss, "l2_loss": l2_loss}


class SampleBuffer:
    """Device-resident training samples fed by the on-device self-play driver.

    ``add(out)`` takes one ``selfplay_move(emit_targets=True)`` result. Moves of
    a game wait in a per-game staging area until the game finishes; then its
    8 x moves samples get their value targets (the final outcome from the
    perspective of the side to move, plane 0 = player - 1) and move into the
    sample store. Capacity is in samples; the oldest are overwritten."""

    def __init__(self, num_games: int, channels: int, capacity: int, max_moves: int = 128,
                 device: torch.device | str | None = None) -> None:
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self.num_games, self.C, self.capacity, self.max_moves = num_games, channels, capacity, max_moves
        d = self.device
        self.features = torch.empty((capacity, channels, 8, 8), dtype=torch.float32, device=d)
        self.policies = torch.empty((capacity, 65), dtype=torch.float32, device=d)
        self.values = torch.empty((capacity,), dtype=torch.float32, device=d)
        self._stage_f = torch.empty((num_games, max_moves, 8, channels, 8, 8), dtype=torch.float32, device=d)
        self._stage_p = torch.empty((num_games, max_moves, 8, 65), dtype=torch.float32, device=d)
        self._moves = torch.zeros(num_games, dtype=torch.int64, device=d)
        self._head = 0
        self.size = 0
        self.games_completed = 0

    def add(self, out: dict[str, torch.Tensor]) -> int:
        """Stage one move of every game; returns the number of samples stored."""
        if "features" not in out:
            raise ValueError("selfplay_move must be called with emit_targets=True")
        actions, finished = out["actions"], out["finished"]
        fin = finished.to(torch.int64)
        if bool(((fin & FIN_OVERFLOW) != 0).any()):
            raise RuntimeError("node pool exhausted: the search no longer matches the reference; "
                               "use a larger node_capacity")
        played = actions >= 0
        if bool(((fin & FIN_NO_TARGETS) != 0)[played].any()):
            raise ValueError("The root node has not been expanded yet.")
        g = torch.nonzero(played).flatten()
        if bool((self._moves[g] >= self.max_moves).any()):
            raise RuntimeError("a game exceeded SampleBuffer.max_moves")
        self._stage_f[g, self._moves[g]] = out["features"][g]
        self._stage_p[g, self._moves[g]] = out["policy"][g]
        self._moves[g] += 1
        done = torch.nonzero((fin & 3) != FIN_NONE).flatten().tolist()
        stored = 0
        for gi in done:
            n = int(self._moves[gi])
            outcome = float(_OUTCOME[int(fin[gi]) & 3])
            f = self._stage_f[gi, :n].reshape(n * 8, self.C, 8, 8)
            black = (f[:, 0, 0, 0] == 0).to(torch.float32)  # plane 0 = player - 1
            v = outcome * (2.0 * black - 1.0)
            self._store(f, self._stage_p[gi, :n].reshape(n * 8, 65), v)
            self._moves[gi] = 0
            self.games_completed += 1
            stored += n * 8
        return stored

    def _store(self, f: torch.Tensor, p: torch.Tensor, v: torch.Tensor) -> None:
        n = f.shape[0]
        idx = (torch.arange(n, device=self.device) + self._head) % self.capacity
        self.features[idx] = f
        self.policies[idx] = p
        self.values[idx] = v
        self._head = (self._head + n) % self.capacity
        self.size = min(self.capacity, self.size + n)


def train_epoch(neural_net: torch.nn.Module, optimizer: torch.optim.Optimizer, features: torch.Tensor,
                policies: torch.Tensor, values: torch.Tensor, batch_size: int, l2_weight: float = 1e-4,
                generator: torch.Generator | None = None) -> dict[str, float]:
    """One pass of train.py:455-521 over (features, policies, values): train
    mode, a shuffled permutation cut into ``len // batch_size`` full batches
    (``drop_last``), per batch zero_grad / forward / ``alphazero_loss`` /
    backward / step; returns the running means of the four losses, as the
    reference does. Tensors may live on the device (``SampleBuffer``) or the
    host; batches are moved to the net's device."""
    neural_net.train()
    dev = next(neural_net.parameters()).device
    n = features.shape[0]
    perm = torch.randperm(n, generator=generator, device="cpu").to(features.device)
    sums = {"total_loss": 0.0, "policy_loss": 0.0, "value_loss": 0.0, "l2_loss": 0.0}
    count = 0
    means: dict[str, float] = {}
    for b in range(n // batch_size):
        idx = perm[b * batch_size:(b + 1) * batch_size]
        x = features[idx].to(dev, torch.float32)
        tp = policies[idx].to(dev, torch.float32)
        tv = values[idx].to(dev, torch.float32)
        optimizer.zero_grad()
        out = neural_net(x)
        losses = alphazero_loss(out["policy"], out["value"], tp, tv, neural_net.parameters(), l2_weight)
        losses["total_loss"].backward()
        optimizer.step()
        count += 1
        for k in sums:
            sums[k] += losses[k].item()
        means = {k: sums[k] / count for k in sums}
    return means


def refresh_native(native_net, neural_net: torch.nn.Module) -> None:
    """Upload the trained weights into the NativeNet the engine searches with
    (BN folded again, eval statistics)."""
    mod = getattr(neural_net, "_orig_mod", neural_net)
    native_net.load_state_dict(mod.state_dict())


__all__ = ["alphazero_loss", "SampleBuffer", "train_epoch", "refresh_native"]

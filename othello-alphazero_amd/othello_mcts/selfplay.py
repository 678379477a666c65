"""Self-play training data from the on-device driver.

``BatchedMCTS.selfplay_move(emit_targets=True)`` plays one move of every game on
the GPU and emits that move's 8-fold targets (mcts.cpp:63-112). ``SelfPlayCollector``
turns the stream of moves into the samples the reference's ``_self_play``
returns (train.py:404-452) once a game is over: per move, 8 feature tensors
``(1+2H, 8, 8)`` and 8 policy tensors ``(65,)``, and the value target of every
sample = the final outcome (+1 black wins / -1 white wins / 0 draw, by disc
count, train.py:438-445) from the perspective of the player to move at that
step. For a game from the initial position that is exactly the reference's
rule "+outcome for step 0, alternate sign every step, passes included"
(train.py:447-450): players alternate every step, passes included. Games that
start from a random opening get the same perspective rule, which the
alternating form would get wrong when white moves first.

The dict returned by ``add`` / ``drain`` has the reference's keys, so it feeds
``_AlphaZeroDataset`` unchanged:
    dataset.features += data["features"]; dataset.policies += data["policies"];
    dataset.values += data["values"]
"""

from __future__ import annotations

import torch

# BatchedMCTS.selfplay_move "finished" codes (csrc/tree.hip k_selfplay_move):
# bits 0-1 outcome of a game that ended with this move, bit 2 no targets were
# written (unexpanded root), bit 3 the game's node pool overflowed
FIN_NONE, FIN_DRAW, FIN_BLACK, FIN_WHITE = 0, 1, 2, 3
FIN_NO_TARGETS, FIN_OVERFLOW = 4, 8
_OUTCOME_BLACK = {FIN_DRAW: 0.0, FIN_BLACK: 1.0, FIN_WHITE: -1.0}


def outcome_for_black(player1_discs: int, player2_discs: int) -> float:
    """+1 / -1 / 0 by the final disc count (train.py:438-445)."""
    b, w = bin(player1_discs).count("1"), bin(player2_discs).count("1")
    return 1.0 if b > w else (-1.0 if b < w else 0.0)


def value_targets_from_outcome(black_to_move: list[bool], player1_discs: int, player2_discs: int) -> list[float]:
    """One value target per move (the reference repeats it for the move's 8
    samples): the final outcome from the perspective of the side to move at that
    step. From the initial position this is train.py:447-450's alternating rule."""
    v = outcome_for_black(player1_discs, player2_discs)
    return [v if b else -v for b in black_to_move]


class SelfPlayCollector:
    """Accumulates selfplay_move outputs per game; completed games become samples.

    ``device``: where returned sample tensors live ("cpu" like the reference's
    dataset, or a CUDA device to keep them in HBM)."""

    def __init__(self, num_games: int, device: str | torch.device = "cpu") -> None:
        self.num_games = num_games
        self.device = torch.device(device)
        self._moves: list[list[tuple[torch.Tensor, torch.Tensor]]] = [[] for _ in range(num_games)]
        self._ready = {"features": [], "policies": [], "values": []}
        self.games_completed = 0

    def add(self, out: dict[str, torch.Tensor]) -> dict[str, list[torch.Tensor]]:
        """Record one selfplay_move(emit_targets=True) result; return (and clear)
        the samples of every game that finished on this move."""
        if "features" not in out:
            raise ValueError("selfplay_move must be called with emit_targets=True")
        actions = out["actions"].to("cpu")
        finished = out["finished"].to("cpu")
        if actions.shape[0] != self.num_games:
            raise ValueError(f"expected {self.num_games} games, got {actions.shape[0]}")
        # the output buffers are reused by the next move: copy this move's targets
        feats = out["features"].to(self.device, copy=True)
        pols = out["policy"].to(self.device, copy=True)
        bad = (finished & FIN_OVERFLOW) != 0
        if bool(bad.any()):
            raise RuntimeError(f"node pool exhausted in game(s) {bad.nonzero().flatten().tolist()}: the search no "
                               "longer matches the reference; use a larger node_capacity")
        no_targets = (finished & FIN_NO_TARGETS) != 0
        if bool((no_targets & (actions >= 0)).any()):
            # the reference's self_play_data raises here (mcts.cpp:69-71)
            raise ValueError("The root node has not been expanded yet.")
        for g in range(self.num_games):
            if int(actions[g]) >= 0:  # a searched, expanded root: targets were written
                self._moves[g].append((feats[g], pols[g]))
            fin = int(finished[g]) & 3
            if fin != FIN_NONE:
                self._finish(g, _OUTCOME_BLACK[fin])
        return self.drain()

    def _finish(self, g: int, outcome_black: float) -> None:
        for f8, p8 in self._moves[g]:
            # plane 0 = player - 1: 0 when black is to move (transformation.h:83-116)
            black_to_move = bool(f8[0, 0, 0, 0] == 0)
            v = outcome_black if black_to_move else -outcome_black
            for t in range(8):
                self._ready["features"].append(f8[t])
                self._ready["policies"].append(p8[t])
                self._ready["values"].append(torch.tensor(v, dtype=torch.float32, device=self.device))
        self._moves[g] = []
        self.games_completed += 1

    def drain(self) -> dict[str, list[torch.Tensor]]:
        out = self._ready
        self._ready = {"features": [], "policies": [], "values": []}
        return out

    def pending_moves(self, game: int) -> int:
        return len(self._moves[game])


def self_play(batched, neural_net, games: int, temperature_moves: int = 12, temperature: float = 1.0,
              opening_moves: int = 0, device: str | torch.device = "cpu",
              moves_per_call: int = 16) -> dict[str, list[torch.Tensor]]:
    """Play until at least ``games`` games have completed across the batch (each
    slot restarts when its game ends) and return their samples in the
    reference's ``_self_play`` format (train.py:404-452). ``opening_moves=0``
    starts every game from the initial position as train.py does.

    With a native net (NativeNet, or a module ``search`` would convert) the
    moves run ``moves_per_call`` at a time through
    ``BatchedMCTS.selfplay_steps`` (free-running games, one enqueue per call:
    the bench's throughput path); per game the moves are those of the
    move-by-move loop (search + selfplay_move), which any other evaluator
    uses, so the samples of the games completed by a given move are the same
    either way. The last call may play up to ``moves_per_call - 1`` moves past
    the one that completed the requested games (their finished games are
    returned too)."""
    from .native import resolve

    col = SelfPlayCollector(batched.num_games, device=device)
    data = {"features": [], "policies": [], "values": []}
    native = moves_per_call > 1 and resolve(neural_net, batched.device.index, batched.config.history_size) is not None
    kw = dict(temperature_moves=temperature_moves, temperature=temperature, opening_moves=opening_moves,
              emit_targets=True)
    while col.games_completed < games:
        if native:
            out = batched.selfplay_steps(neural_net, moves_per_call, keep_all=True, **kw)
            moves = [{k: v[i] for k, v in out.items()} for i in range(moves_per_call)]
        else:
            batched.search(neural_net)
            moves = [batched.selfplay_move(**kw)]
        for o in moves:
            got = col.add(o)
            for k in data:
                data[k] += got[k]
    return data


__all__ = ["SelfPlayCollector", "self_play", "outcome_for_black", "value_targets_from_outcome",
           "FIN_NO_TARGETS", "FIN_OVERFLOW", "FIN_NONE", "FIN_DRAW", "FIN_BLACK", "FIN_WHITE"]

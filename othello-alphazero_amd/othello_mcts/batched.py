"""Batched multi-game search: G independent games on one GPU.

The reference searches one game per ``MCTS`` object and plays games one after
another (train.py:394-398). ``BatchedMCTS`` keeps G game trees in HBM and
advances all of them with the same kernel launches (csrc/tree.hip), the NN
evaluating G * num_threads * batch_size leaves per launch. With G = 1 it is
the reference's single-game search; every game follows exactly the
single-game semantics (tested against the oracle game by game).
"""

from __future__ import annotations

import torch

from ._othello_mcts_impl import SearchConfig, _Engine
from .native import NativeNet, resolve


def default_node_capacity(num_simulations: int) -> int:
    """Power of two >= 64 searches x num_simulations x 12 nodes, in [2^16, 2^22]
    (observed: ~8.5 children per expansion, games of <= 64 plies; 800 sims ->
    2^20 nodes = 64 MB per game, 1600 sims -> 2^21)."""
    need = 64 * max(1, num_simulations) * 12
    cap = 1 << 16
    while cap < need and cap < (1 << 22):
        cap <<= 1
    return cap


class BatchedMCTS:
    def __init__(
        self,
        num_games: int,
        history_size: int = 8,
        num_simulations: int = 800,
        num_threads: int = 2,
        batch_size: int = 16,
        c_puct_base: float = 20000.0,
        c_puct_init: float = 2.5,
        dirichlet_epsilon: float = 0.25,
        dirichlet_alpha: float = 0.5,
        device: int | None = None,
        seed: int = 0,
        node_capacity: int = 0,
    ) -> None:
        """node_capacity: nodes per game (0 = sized from num_simulations: a whole
        game of 64 searches at ~12 new nodes per simulation, 2^16..2^22). Nodes are
        reclaimed when a game restarts; running out raises (check_health)."""
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device)
        self.config = SearchConfig(history_size, num_simulations, num_threads, batch_size, c_puct_base,
                                   c_puct_init, dirichlet_epsilon, dirichlet_alpha)
        if node_capacity == 0:
            node_capacity = default_node_capacity(num_simulations)
        self.node_capacity = node_capacity
        self.engine = _Engine(device, num_games, node_capacity, self.config, seed)
        self.num_games = num_games
        self._actions = torch.empty(num_games, dtype=torch.int32, device=self.device)
        self._finished = torch.empty(num_games, dtype=torch.int32, device=self.device)
        C = 1 + 2 * history_size
        self._targets_f = None
        self._targets_p = None
        self._C = C

    @property
    def rows_per_step(self) -> int:
        return self.num_games * self.config.num_threads * self.config.batch_size

    def _stream(self) -> int:
        s = torch.cuda.current_stream(self.device).cuda_stream
        self.engine.set_stream(s)
        return s

    def search(self, neural_net, sync: bool = True):
        """Run num_simulations for every active game. Returns (simulations, nn_rows).

        With the native net and ``sync=False`` the search is only enqueued on the
        engine's stream (returns None): a self-play loop then queues the next
        move's kernels while the GPU still runs this one's."""
        self._stream()
        nat = resolve(neural_net, self.device.index, self.config.history_size)
        if nat is not None:
            r = self.engine.search(nat.handle, sync)
            if sync:
                self.engine.check_health()  # raises if a node pool ran out
            return r
        # external evaluator: one call per step over all G * L rows. Each select
        # backs up the previous round thread by thread (the reference's
        # interleaving, csrc/tree.hip k_tree); one backup closes the search.
        rows = self.rows_per_step
        feat = torch.empty((rows, self._C, 8, 8), dtype=torch.float32, device=self.device)
        sims0, evals0 = self.engine.work_counters()
        steps = self.engine.search_begin()
        for _ in range(steps):
            self.engine.select()
            # every row goes to the evaluator; rows of terminal leaves and of
            # threads with no batch waiting this round are never read back
            self.engine.features(feat.data_ptr(), 0, rows)
            out = neural_net(feat)
            pol = out["policy"].detach().to(self.device, torch.float32).contiguous()
            val = out["value"].detach().to(self.device, torch.float32).contiguous()
            self.engine.set_evaluation(pol.data_ptr(), val.data_ptr(), 0, rows)
        self.engine.backup()
        self.engine.check_health()
        sims1, evals1 = self.engine.work_counters()
        # simulations = leaf selections; evaluations = rows of non-terminal
        # leaves (terminal ones need no NN, search_thread.cpp:88-90)
        return sims1 - sims0, evals1 - evals0

    def check_health(self) -> None:
        """Raise RuntimeError if any game's node pool ran out or a descent hit
        the depth cap (waits for the engine's stream). Asynchronous searches
        (sync=False) are checked here or by SelfPlayCollector."""
        self._stream()
        self.engine.check_health()

    def reset(self, game: int = -1, seed: int = 0) -> None:
        self._stream()
        self.engine.reset(game, seed)

    def random_openings(self, max_moves: int = 8, seed: int = 0) -> None:
        self._stream()
        self.engine.random_openings(max_moves, seed)

    def root_info(self, game: int) -> dict:
        self._stream()
        return self.engine.root_info(game)

    def visit_counts(self, game: int) -> list[int]:
        return self.root_info(game)["visit_counts"]

    def mean_action_values(self, game: int) -> list[float]:
        return self.root_info(game)["mean_action_values"]

    def root_stats(self) -> tuple[torch.Tensor, torch.Tensor]:
        """(visits, q) of every game's root children, (G, 65) indexed by action."""
        self._stream()
        v = torch.empty((self.num_games, 65), dtype=torch.int32, device=self.device)
        q = torch.empty((self.num_games, 65), dtype=torch.float32, device=self.device)
        self.engine.root_stats(v.data_ptr(), q.data_ptr(), 0)
        return v, q

    def self_play_data(self, game: int):
        self._stream()
        f, p = self.engine.self_play_data(game)
        return {"features": list(torch.from_numpy(f)), "policy": list(torch.from_numpy(p))}

    def apply_action(self, game: int, action: int) -> None:
        self._stream()
        self.engine.apply_action(game, action)

    def apply_actions(self, actions: torch.Tensor) -> None:
        """actions: (G,) int32 on the engine's device, -1 = leave the game."""
        self._stream()
        a = actions.to(self.device, torch.int32).contiguous()
        self.engine.apply_actions(a.data_ptr())

    def selfplay_move(self, temperature_moves: int = 12, temperature: float = 1.0, opening_moves: int = 0,
                      emit_targets: bool = False) -> dict[str, torch.Tensor]:
        """One self-play move for every game (train.py:404-452 on device): choose the
        move from the root visits, (optionally) emit the 8-fold targets, apply it, and
        restart finished games from a random opening. Returns device tensors."""
        self._stream()
        if emit_targets and self._targets_f is None:
            self._targets_f = torch.empty((self.num_games, 8, self._C, 8, 8), dtype=torch.float32,
                                          device=self.device)
            self._targets_p = torch.empty((self.num_games, 8, 65), dtype=torch.float32, device=self.device)
        f = self._targets_f.data_ptr() if emit_targets else 0
        p = self._targets_p.data_ptr() if emit_targets else 0
        self.engine.selfplay_move(temperature_moves, temperature, opening_moves, emit_targets,
                                  self._actions.data_ptr(), self._finished.data_ptr(), f, p)
        out = {"actions": self._actions, "finished": self._finished}
        if emit_targets:
            out["features"] = self._targets_f
            out["policy"] = self._targets_p
        return out

    def selfplay_steps(self, neural_net, n_moves: int, temperature_moves: int = 12, temperature: float = 1.0,
                       opening_moves: int = 0, emit_targets: bool = False,
                       keep_all: bool = True) -> dict[str, torch.Tensor]:
        """n_moves x (search(net) + selfplay_move(...)) in one enqueue, same results
        move for move; each pipeline group chains its searches and moves on its own
        stream, so the per-move join disappears (oamd_engine_selfplay_steps).
        keep_all: outputs shaped (n_moves, G, ...); else only the last move's
        (G, ...), every move writing the same buffers. Native net (or a module
        search() would convert) only."""
        self._stream()
        net = resolve(neural_net, self.device.index, self.config.history_size)
        if net is None:
            raise TypeError("selfplay_steps needs a NativeNet (or an eval-mode AlphaZeroNet)")
        n = max(0, int(n_moves))
        lead = (n,) if keep_all else ()
        actions = torch.empty(lead + (self.num_games,), dtype=torch.int32, device=self.device)
        finished = torch.empty_like(actions)
        feat = pol = None
        if emit_targets:
            feat = torch.empty(lead + (self.num_games, 8, self._C, 8, 8), dtype=torch.float32, device=self.device)
            pol = torch.empty(lead + (self.num_games, 8, 65), dtype=torch.float32, device=self.device)
        self.engine.selfplay_steps(net.handle, n, temperature_moves, temperature, opening_moves, emit_targets,
                                   keep_all, actions.data_ptr(), finished.data_ptr(),
                                   feat.data_ptr() if feat is not None else 0,
                                   pol.data_ptr() if pol is not None else 0)
        out = {"actions": actions, "finished": finished}
        if emit_targets:
            out["features"] = feat
            out["policy"] = pol
        return out


__all__ = ["BatchedMCTS", "NativeNet"]

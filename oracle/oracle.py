"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper around oracle/_build/liboracle.so (the plain-C restatement of
the reference othello_mcts path, see omcts_oracle.h). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module,
as the checker / the CPU baseline. The product never imports it.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "liboracle.so"


def build(force: bool = False) -> Path:
    if force or not LIB_PATH.exists() or (
        LIB_PATH.stat().st_mtime < (HERE / "omcts_oracle.c").stat().st_mtime
    ):
        subprocess.run(["make", "-s", "-C", str(HERE), "all"], check=True)
    return LIB_PATH


class CPos(ctypes.Structure):
    _fields_ = [
        ("player", ctypes.c_int32),
        ("p1", ctypes.c_uint64),
        ("p2", ctypes.c_uint64),
        ("legal", ctypes.c_uint64),
        ("next_legal", ctypes.c_uint64),
    ]

    def tuple(self):
        return (self.player, self.p1, self.p2, self.legal, self.next_legal)


NN_FN = ctypes.CFUNCTYPE(
    None,
    ctypes.c_void_p,
    ctypes.POINTER(ctypes.c_float),
    ctypes.c_int,
    ctypes.c_int,
    ctypes.POINTER(ctypes.c_float),
    ctypes.POINTER(ctypes.c_float),
)

_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(str(LIB_PATH))
        u64, i32, f32, vp = ctypes.c_uint64, ctypes.c_int, ctypes.c_float, ctypes.c_void_p
        P = ctypes.POINTER
        sig = {
            "orc_get_legal_moves": (u64, [u64, u64]),
            "orc_get_flips": (u64, [u64, u64, u64]),
            "orc_initial_position": (None, [P(CPos)]),
            "orc_apply_action": (None, [P(CPos), i32, P(CPos)]),
            "orc_legal_actions": (i32, [P(CPos), P(ctypes.c_int32)]),
            "orc_transform_action": (i32, [i32, i32]),
            "orc_legal_moves_n": (None, [vp, vp, vp, ctypes.c_int64]),
            "orc_flips_n": (None, [vp, vp, vp, vp, ctypes.c_int64]),
            "orc_apply_action_n": (None, [vp] * 11 + [ctypes.c_int64]),
            "orc_features": (None, [P(CPos), i32, i32, i32, P(f32)]),
            "orc_mix64": (u64, [u64]),
            "orc_stream_key": (u64, [u64, u64, ctypes.c_uint32]),
            "orc_uniform": (f32, [u64, ctypes.c_uint32]),
            "orc_logf": (f32, [f32]),
            "orc_expf": (f32, [f32]),
            "orc_gamma": (f32, [u64, f32]),
            "orc_cos2pi_sq": (f32, [f32]),
            "orc_mcts_create": (vp, [i32, i32, i32, i32, f32, f32, f32, f32, u64]),
            "orc_mcts_destroy": (None, [vp]),
            "orc_mcts_reset_position": (None, [vp]),
            "orc_mcts_reset_chain": (None, [vp, P(CPos), i32]),
            "orc_mcts_position": (None, [vp, P(CPos)]),
            "orc_mcts_search": (i32, [vp, NN_FN, vp]),
            "orc_mcts_num_children": (i32, [vp]),
            "orc_mcts_visit_counts": (None, [vp, P(ctypes.c_int32)]),
            "orc_mcts_mean_action_values": (None, [vp, P(f32)]),
            "orc_mcts_root_visit_count": (ctypes.c_int32, [vp]),
            "orc_mcts_self_play_data": (i32, [vp, P(f32), P(f32)]),
            "orc_mcts_apply_action": (i32, [vp, i32]),
            "orc_mcts_node_count": (i32, [vp]),
            "orc_mcts_events": (u64, [vp]),
            "orc_mcts_selfplay_action": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.c_float]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


# ---------------------------------------------------------------- bitboards
def get_legal_moves(me: int, opp: int) -> int:
    return lib().orc_get_legal_moves(me, opp)


def get_flips(move: int, me: int, opp: int) -> int:
    return lib().orc_get_flips(move, me, opp)


def initial_position() -> CPos:
    p = CPos()
    lib().orc_initial_position(ctypes.byref(p))
    return p


def apply_action(p: CPos, action: int) -> CPos:
    out = CPos()
    lib().orc_apply_action(ctypes.byref(p), action, ctypes.byref(out))
    return out


def legal_actions(p: CPos) -> list[int]:
    buf = (ctypes.c_int32 * 65)()
    n = lib().orc_legal_actions(ctypes.byref(p), buf)
    return list(buf[:n])


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


def legal_moves_n(me: np.ndarray, opp: np.ndarray) -> np.ndarray:
    me = np.ascontiguousarray(me, np.uint64)
    opp = np.ascontiguousarray(opp, np.uint64)
    out = np.empty_like(me)
    lib().orc_legal_moves_n(_p(me), _p(opp), _p(out), me.size)
    return out


def flips_n(mv: np.ndarray, me: np.ndarray, opp: np.ndarray) -> np.ndarray:
    mv, me, opp = (np.ascontiguousarray(x, np.uint64) for x in (mv, me, opp))
    out = np.empty_like(me)
    lib().orc_flips_n(_p(mv), _p(me), _p(opp), _p(out), me.size)
    return out


def apply_action_n(player, p1, p2, legal, next_legal, action):
    player = np.ascontiguousarray(player, np.int32)
    p1, p2, legal, next_legal = (np.ascontiguousarray(x, np.uint64) for x in (p1, p2, legal, next_legal))
    action = np.ascontiguousarray(action, np.int32)
    n = player.size
    out = [np.empty(n, np.int32)] + [np.empty(n, np.uint64) for _ in range(4)]
    lib().orc_apply_action_n(_p(player), _p(p1), _p(p2), _p(legal), _p(next_legal), _p(action),
                             *(_p(x) for x in out), n)
    return out


def transform_action(a: int, t: int) -> int:
    return lib().orc_transform_action(a, t)


def features(chain: list[CPos], history_size: int, t: int) -> np.ndarray:
    arr = (CPos * max(1, len(chain)))(*chain)
    out = np.zeros((1 + 2 * history_size) * 64, dtype=np.float32)
    lib().orc_features(
        arr, len(chain), history_size, t, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    )
    return out.reshape(1 + 2 * history_size, 8, 8)


# ---------------------------------------------------------------- MCTS
class OracleMCTS:
    """Single-game oracle MCTS with the reference's parameter names and defaults
    (othello_mcts.cpp:89-112)."""

    def __init__(
        self,
        history_size: int = 4,
        num_simulations: int = 800,
        num_threads: int = 2,
        batch_size: int = 16,
        c_puct_base: float = 20000.0,
        c_puct_init: float = 2.5,
        dirichlet_epsilon: float = 0.25,
        dirichlet_alpha: float = 0.5,
        game_key: int = 0,
    ) -> None:
        self.history_size = history_size
        self._h = lib().orc_mcts_create(
            history_size,
            num_simulations,
            num_threads,
            batch_size,
            c_puct_base,
            c_puct_init,
            dirichlet_epsilon,
            dirichlet_alpha,
            game_key,
        )

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.orc_mcts_destroy(h)
            self._h = None

    def reset_position(self) -> None:
        lib().orc_mcts_reset_position(self._h)

    def reset_chain(self, chain: list[CPos]) -> None:
        arr = (CPos * len(chain))(*chain)
        lib().orc_mcts_reset_chain(self._h, arr, len(chain))

    def position(self) -> CPos:
        p = CPos()
        lib().orc_mcts_position(self._h, ctypes.byref(p))
        return p

    def search(self, nn) -> int:
        """nn(features: np.ndarray (rows, C, 8, 8) float32) -> (policy (rows,65), value (rows,))."""

        err: list[BaseException] = []

        def cb(_user, feat, rows, channels, pol, val):
            try:
                f = np.ctypeslib.as_array(feat, shape=(rows, channels, 8, 8))
                p, v = nn(f)
                np.ctypeslib.as_array(pol, shape=(rows, 65))[:] = np.asarray(p, np.float32)
                np.ctypeslib.as_array(val, shape=(rows,))[:] = np.asarray(v, np.float32)
            except BaseException as e:  # noqa: BLE001 - re-raised below
                err.append(e)

        fn = NN_FN(cb)
        n = lib().orc_mcts_search(self._h, fn, None)
        if err:
            raise err[0]
        return n

    def visit_counts(self) -> list[int]:
        n = lib().orc_mcts_num_children(self._h)
        buf = (ctypes.c_int32 * max(n, 1))()
        lib().orc_mcts_visit_counts(self._h, buf)
        return list(buf[:n])

    def mean_action_values(self) -> list[float]:
        n = lib().orc_mcts_num_children(self._h)
        buf = (ctypes.c_float * max(n, 1))()
        lib().orc_mcts_mean_action_values(self._h, buf)
        return list(buf[:n])

    def root_visit_count(self) -> int:
        return lib().orc_mcts_root_visit_count(self._h)

    def self_play_data(self):
        C = 1 + 2 * self.history_size
        f = np.zeros((8, C, 8, 8), np.float32)
        p = np.zeros((8, 65), np.float32)
        rc = lib().orc_mcts_self_play_data(
            self._h,
            f.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
            p.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
        )
        if rc == 1:
            raise ValueError("Self-play data cannot be generated from a terminal position.")
        if rc == 2:
            raise ValueError("The root node has not been expanded yet.")
        return f, p

    def apply_action(self, action: int) -> None:
        rc = lib().orc_mcts_apply_action(self._h, action)
        if rc == -1:
            raise IndexError(f"Expected 0 <= action < 65, but got {action}.")
        if rc == -2:
            raise ValueError(f"{action} is not a legal action.")
        if rc == -3:
            raise ValueError("Pass is not allowed in a terminal position.")
        if rc == -4:
            raise ValueError("Pass is not allowed when there are legal moves.")

    def node_count(self) -> int:
        return lib().orc_mcts_node_count(self._h)

    def events(self) -> int:
        return lib().orc_mcts_events(self._h)

    def selfplay_action(self, ply: int, temperature_moves: int = 12, temperature: float = 1.0) -> int:
        """train.py:421-430's choice as the on-device driver draws it (consumes one event)."""
        return lib().orc_mcts_selfplay_action(self._h, ply, temperature_moves, temperature)


# ---------------------------------------------------------------- stub nets
def equivariant_stub(features: np.ndarray):
    """SURVEY.md Appendix B.3 stub net (per-square policy, global value), torch
    fp32 on CPU exactly as the survey's known-answer runs computed it."""
    import torch

    x = torch.from_numpy(np.ascontiguousarray(features))
    C = x.shape[1]
    w = torch.linspace(-1, 1, C)
    sq = (x * w.view(1, C, 1, 1)).sum(dim=1).flatten(1)
    logits = torch.cat([sq, torch.full((x.shape[0], 1), -2.0)], dim=1)
    policy = torch.softmax(logits, dim=1)
    value = torch.tanh(sq.mean(dim=1) + 0.1 * x[:, 0].flatten(1).mean(dim=1))
    return policy.numpy(), value.numpy()


def uniform_stub(features: np.ndarray):
    n = features.shape[0]
    return np.full((n, 65), 1.0 / 65.0, np.float32), np.zeros(n, np.float32)


if __name__ == "__main__":  # pragma: no cover
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    m = OracleMCTS(history_size=4, num_threads=1, batch_size=16, dirichlet_epsilon=0.0)
    m.search(equivariant_stub)
    print(m.visit_counts())

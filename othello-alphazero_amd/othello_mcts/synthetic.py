"""Synthetic inputs for benchmarks and parity tests.

* ``alphazero_state_dict`` — seeded random weights for the reference's
  ``AlphaZeroNet`` (python/othello_alphazero/neural_net.py:138-172) with the
  reference's exact ``state_dict`` keys. Values come from a
  portable counter-based generator (splitmix64) so fixtures generated in one
  place can be regenerated anywhere without shipping weight files. Scales
  follow torch's default init (uniform ±1/sqrt(fan_in)); BatchNorm running
  statistics are perturbed away from identity so BN folding is exercised.
* ``random_openings`` — the SURVEY.md §8(d) opening spec: game g starts from
  the initial position plus k_g ~ U{0..8} uniformly random legal moves.
"""

from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def portable_uniform(seed: int, stream: int, n: int) -> np.ndarray:
    """n float64 uniforms in [0, 1) from stream ``stream`` of ``seed``."""
    with np.errstate(over="ignore"):
        key = _mix64(np.array([seed], np.uint64) ^ (np.uint64(stream) * np.uint64(0xD1B54A32D192ED03)))
        idx = np.arange(1, n + 1, dtype=np.uint64)
        x = _mix64(key + idx * _GOLDEN)
    return (x >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def alphazero_state_dict(
    seed: int,
    in_channels: int = 17,
    conv_channels: int = 128,
    num_residual_blocks: int = 9,
    value_head_hidden_channels: int = 128,
    num_squares: int = 64,
    num_actions: int = 65,
) -> dict[str, np.ndarray]:
    """Seeded float32 weights keyed exactly like AlphaZeroNet.state_dict()."""
    C = conv_channels
    shapes: list[tuple[str, tuple[int, ...], str, int]] = []

    def conv(prefix: str, cin: int, cout: int, k: int) -> None:
        fan_in = cin * k * k
        shapes.append((f"{prefix}.weight", (cout, cin, k, k), "fan", fan_in))
        shapes.append((f"{prefix}.bias", (cout,), "fan", fan_in))

    def bn(prefix: str, c: int) -> None:
        shapes.append((f"{prefix}.weight", (c,), "gamma", 0))
        shapes.append((f"{prefix}.bias", (c,), "beta", 0))
        shapes.append((f"{prefix}.running_mean", (c,), "mean", 0))
        shapes.append((f"{prefix}.running_var", (c,), "var", 0))
        shapes.append((f"{prefix}.num_batches_tracked", (), "count", 0))

    def linear(prefix: str, fin: int, fout: int) -> None:
        shapes.append((f"{prefix}.weight", (fout, fin), "fan", fin))
        shapes.append((f"{prefix}.bias", (fout,), "fan", fin))

    conv("conv_block.conv", in_channels, C, 3)
    bn("conv_block.norm", C)
    for i in range(num_residual_blocks):
        conv(f"residual_blocks.{i}.conv1", C, C, 3)
        bn(f"residual_blocks.{i}.norm1", C)
        conv(f"residual_blocks.{i}.conv2", C, C, 3)
        bn(f"residual_blocks.{i}.norm2", C)
    conv("policy_head.conv", C, 2, 1)
    bn("policy_head.norm", 2)
    linear("policy_head.linear", 2 * num_squares, num_actions)
    conv("value_head.conv", C, 1, 1)
    bn("value_head.norm", 1)
    linear("value_head.linear1", num_squares, value_head_hidden_channels)
    linear("value_head.linear2", value_head_hidden_channels, 1)

    out: dict[str, np.ndarray] = {}
    for stream, (name, shape, kind, fan) in enumerate(shapes):
        n = int(np.prod(shape)) if shape else 1
        u = portable_uniform(seed, stream, n)
        if kind == "fan":
            b = 1.0 / np.sqrt(fan)
            v = (2.0 * u - 1.0) * b
        elif kind == "gamma":
            v = 0.5 + u
        elif kind == "beta":
            v = (2.0 * u - 1.0) * 0.1
        elif kind == "mean":
            v = (2.0 * u - 1.0) * 0.2
        elif kind == "var":
            v = 0.5 + u
        else:  # num_batches_tracked
            out[name] = np.array(0, dtype=np.int64)
            continue
        out[name] = v.astype(np.float32).reshape(shape)
    return out


def net_config_from_state_dict(sd) -> dict[str, int]:
    """Recover AlphaZeroNet(**config) from a state_dict (numpy or torch)."""
    w0 = sd["conv_block.conv.weight"]
    blocks = 0
    while f"residual_blocks.{blocks}.conv1.weight" in sd:
        blocks += 1
    return {
        "in_channels": int(w0.shape[1]),
        "num_squares": int(sd["value_head.linear1.weight"].shape[1]),
        "num_actions": int(sd["policy_head.linear.weight"].shape[0]),
        "conv_channels": int(w0.shape[0]),
        "num_residual_blocks": blocks,
        "value_head_hidden_channels": int(sd["value_head.linear1.weight"].shape[0]),
    }


# ------------------------------------------------------------- openings
def _splitmix_stream(seed: int):
    state = seed & 0xFFFFFFFFFFFFFFFF
    while True:
        state = (state + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        yield z ^ (z >> 31)


def random_opening_actions(seed: int, max_moves: int = 8, position_cls=None) -> list[int]:
    """Actions of one random opening: k ~ U{0..max_moves}
    uniformly random legal actions from the initial position (stops early at a
    terminal position, which cannot happen within 8 plies)."""
    if position_cls is None:
        from . import Position as position_cls  # noqa: N813
    rng = _splitmix_stream(seed)
    k = next(rng) % (max_moves + 1)
    p = position_cls.initial_position()
    actions = []
    for _ in range(k):
        if p.is_terminal():
            break
        legal = p.legal_actions()
        a = legal[next(rng) % len(legal)]
        actions.append(a)
        p = p.apply_action(a)
    return actions

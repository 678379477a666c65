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


# ------------------------------------------------- live (trained-like) nets
def calibration_features(n: int, history_size: int, seed: int, position_cls=None) -> np.ndarray:
    """Feature planes (n, 1+2H, 8, 8) of `n` real positions: seeded random games
    of 0-57 plies from the initial position, each with its history, laid out
    like positions_to_features (transformation.h:83-116) untransformed (a
    calibration batch: BN statistics do not depend on the symmetry)."""
    if position_cls is None:
        from . import Position as position_cls  # noqa: N813
    rng = _splitmix_stream(seed ^ 0x5CA1AB1E)
    C = 1 + 2 * history_size
    out = np.zeros((n, C, 64), np.float32)
    bits = np.array([1 << (63 - s) for s in range(64)], dtype=np.uint64)
    for i in range(n):
        chain = [position_cls.initial_position()]
        for _ in range(next(rng) % 58):
            p = chain[-1]
            if p.is_terminal():
                break
            acts = p.legal_actions()
            chain.append(p.apply_action(acts[next(rng) % len(acts)]))
        if chain[-1].is_terminal():
            chain.pop()
        leaf = chain[-1]
        out[i, 0] = float(leaf.player() - 1)
        for h, p in enumerate(reversed(chain[-history_size:])):
            out[i, 1 + 2 * h] = (np.uint64(p.player1_discs()) & bits) != 0
            out[i, 2 + 2 * h] = (np.uint64(p.player2_discs()) & bits) != 0
    return out.reshape(n, C, 8, 8)


def live_state_dict(
    seed: int,
    in_channels: int = 17,
    conv_channels: int = 128,
    num_residual_blocks: int = 9,
    value_head_hidden_channels: int = 128,
    policy: str = "random",
    policy_sharpness: float = 1.0,
    value_spread: float = 0.75,
    calibration_positions: int = 96,
    position_cls=None,
) -> dict[str, np.ndarray]:
    """Seeded weights of a net whose outputs depend on its input, like a
    trained one's (torch-default random init at 10 blocks forgets
    its input — each conv shrinks the signal ~6x, so the tower's output is its
    biases, the value constant and the priors uniform).

    * Convolutions: He-scaled (variance 2 / fan_in) uniform weights.
    * BatchNorm running statistics set the way training leaves them: the batch
      statistics of each BN's input over `calibration_positions` real
      positions (calibration_features), computed in float64 layer by layer
      through the reference's forward (neural_net.py:9-128); gamma / beta stay
      seeded (0.5-1.5 / +-0.1).
    * Value head: linear2 rescaled so that its pre-tanh output has standard
      deviation `value_spread` and mean 0 over the calibration batch.
    * policy="random": the policy linear layer as seeded, logits scaled by
      `policy_sharpness`.
      policy="frontier": priors peaked on plausible moves, like a trained
      net's. Two tower channels carry, per empty square, the number of
      neighbouring discs of the side NOT to move (conv0's channels 0 / 1 for
      black / white to move, identity through every residual block:
      norm2's gamma = beta = 0 there); the policy head's first channel sums
      them and its linear layer reads that square's count times
      `policy_sharpness` on top of the seeded weights (x 0.5). Legal moves
      are a subset of these frontier squares.
    Deterministic for a seed: the statistics are rounded to float32 from
    float64 sums."""
    import torch
    import torch.nn.functional as F

    C, R, hid = conv_channels, num_residual_blocks, value_head_hidden_channels
    sd = {k: np.array(v, copy=True) for k, v in
          alphazero_state_dict(seed, in_channels, C, R, hid).items()}
    for k, v in sd.items():  # He scale: +-1/sqrt(fan) uniform -> +-sqrt(6/fan)
        if v.ndim == 4 and k.endswith(".weight") and not k.startswith(("policy_head", "value_head")):
            sd[k] = (v * np.sqrt(6.0)).astype(np.float32)
    frontier = policy == "frontier"
    if policy not in ("random", "frontier"):
        raise ValueError(f"policy must be 'random' or 'frontier', got {policy!r}")
    if frontier:
        w = sd["conv_block.conv.weight"]
        b = sd["conv_block.conv.bias"]
        w[0:2] = 0.0
        nbr = np.ones((3, 3), np.float32)
        nbr[1, 1] = 0.0
        # ch 0: black to move (plane 0 = 0), count white (plane 2) neighbours
        w[0, 2] = nbr
        w[0, 1, 1, 1] = w[0, 2, 1, 1] = -9.0
        w[0, 0, 1, 1] = -9.0
        b[0] = 0.0
        # ch 1: white to move (plane 0 = 1), count black (plane 1) neighbours
        w[1, 1] = nbr
        w[1, 1, 1, 1] = w[1, 2, 1, 1] = -9.0
        w[1, 0, 1, 1] = 9.0
        b[1] = -9.0
    x = torch.from_numpy(calibration_features(calibration_positions, (in_channels - 1) // 2, seed,
                                              position_cls)).double()
    t = {k: torch.from_numpy(v).double() for k, v in sd.items() if v.ndim > 0}

    def bn(h, p, keep=()):
        mean = h.mean(dim=(0, 2, 3))
        var = h.var(dim=(0, 2, 3), unbiased=False)
        for c in keep:  # carried channels: identity BN
            mean[c] = 0.0
            var[c] = 1.0
            t[p + ".weight"][c] = 1.0
            t[p + ".bias"][c] = 0.0
        t[p + ".running_mean"] = mean.float().double()
        t[p + ".running_var"] = var.float().double()
        sd[p + ".running_mean"] = mean.float().numpy()
        sd[p + ".running_var"] = var.float().numpy()
        sd[p + ".weight"] = t[p + ".weight"].float().numpy()
        sd[p + ".bias"] = t[p + ".bias"].float().numpy()
        return F.batch_norm(h, t[p + ".running_mean"], t[p + ".running_var"], t[p + ".weight"], t[p + ".bias"],
                            training=False, eps=1e-5)

    def conv(h, p, pad):
        return F.conv2d(h, t[p + ".weight"], t[p + ".bias"], padding=pad)

    carried = (0, 1) if frontier else ()
    h = F.relu(bn(conv(x, "conv_block.conv", 1), "conv_block.norm", carried))
    for i in range(R):
        p = f"residual_blocks.{i}"
        a = F.relu(bn(conv(h, p + ".conv1", 1), p + ".norm1"))
        if frontier:
            t[p + ".norm2.weight"][0:2] = 0.0
            t[p + ".norm2.bias"][0:2] = 0.0
        h = F.relu(bn(conv(a, p + ".conv2", 1), p + ".norm2") + h)
    if frontier:
        pw = t["policy_head.conv.weight"]
        pw[0] = 0.0
        pw[0, 0:2] = 1.0
        t["policy_head.conv.bias"][0] = 0.0
        sd["policy_head.conv.weight"] = pw.float().numpy()
        sd["policy_head.conv.bias"] = t["policy_head.conv.bias"].float().numpy()
    bn(conv(h, "policy_head.conv", 0), "policy_head.norm", (0,) if frontier else ())
    lw = sd["policy_head.linear.weight"]
    if frontier:
        lw = lw * 0.5
        lw[np.arange(64), np.arange(64)] += policy_sharpness  # channel 0, square a -> action a
        sd["policy_head.linear.bias"][64] = -2.0  # pass: only ever a single child
    else:
        lw = lw * policy_sharpness
        sd["policy_head.linear.bias"] = sd["policy_head.linear.bias"] * policy_sharpness
    sd["policy_head.linear.weight"] = lw.astype(np.float32)
    v = F.relu(bn(conv(h, "value_head.conv", 0), "value_head.norm"))
    v = F.relu(F.linear(v.flatten(1), t["value_head.linear1.weight"], t["value_head.linear1.bias"]))
    z = F.linear(v, t["value_head.linear2.weight"])[:, 0]
    s = value_spread / max(float(z.std(unbiased=False)), 1e-12)
    sd["value_head.linear2.weight"] = (sd["value_head.linear2.weight"] * s).astype(np.float32)
    sd["value_head.linear2.bias"] = np.array([-float(z.mean()) * s], np.float32)
    for k in sd:
        if k.endswith("num_batches_tracked"):
            sd[k] = np.array(0, dtype=np.int64)
        else:
            sd[k] = np.ascontiguousarray(sd[k], dtype=np.float32)
    return sd


# ------------------------------------------------- self-play trained net
BENCH_NETS = __import__("pathlib").Path(__file__).resolve().parents[2] / "bench_nets"


def selfplay_state_dict(name: str = "selfplay_128x10b_h8") -> dict[str, np.ndarray]:
    """A 128x10b net trained by this package's own self-play loop
    (tools/selfplay_train.py: 15k games of 800-sim self-play from a live init,
    the reference's loss and SGD settings; bench_nets/NAME.json is its log),
    stored as float16 with the reference's state_dict keys. Loaded without
    unpickling (numpy.load, allow_pickle=False). Its priors sit on legal moves
    (mass 0.99) and its value tracks game outcomes, like a trained net's."""
    z = np.load(BENCH_NETS / f"{name}.npz", allow_pickle=False)
    return {k: (np.array(0, dtype=np.int64) if k.endswith("num_batches_tracked")
                else np.ascontiguousarray(z[k], dtype=np.float32)) for k in z.files}

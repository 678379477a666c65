"""The benched synthetic nets are live.

Round 1-4's seeded torch-default init forgot its input after 10 blocks (each
conv shrinks the signal ~6x): the value head output a constant and the priors
were within 0.02 nats of uniform, so the headline searched shallow
breadth-first trees. `live_state_dict` (He-scaled convs, BN statistics of real
positions, a value head spread over [-1, 1]) is what bench.py runs; the
deep_tree sub-record runs its frontier variant, whose priors are peaked like a
trained net's. Checked here through the fp32 restatement of the reference's
AlphaZeroNet (oracle/resnet_ref.py, pinned by the reference's own outputs in
test_oracle_golden.py) on 256 real positions (random games, their histories,
random symmetries; tests/ref_fixtures.real_features)."""

import sys
from pathlib import Path

import numpy as np
import pytest
import torch

import resnet_ref
from ref_fixtures import real_features

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
import oracle as O  # noqa: E402


def _legal_mask(x: np.ndarray) -> np.ndarray:
    m = np.zeros((len(x), 65), bool)
    bits = [1 << (63 - s) for s in range(64)]
    for i, f in enumerate(x):
        b = sum(bits[s] for s in range(64) if f[1].flat[s] > 0)
        w = sum(bits[s] for s in range(64) if f[2].flat[s] > 0)
        me, opp = (w, b) if f[0, 0, 0] > 0 else (b, w)
        lm = O.get_legal_moves(me, opp)
        m[i, :64] = [(lm >> (63 - s)) & 1 == 1 for s in range(64)]
        m[i, 64] = lm == 0
    return m


@pytest.fixture(scope="module")
def positions():
    x = real_features(256, 8, 7)
    return torch.from_numpy(x), _legal_mask(x)


def _outputs(sd, x):
    out = resnet_ref.forward({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, x)
    return out["policy"].numpy(), out["value"].numpy()


# every benched net: configs[1] / [4] (128x10b, bf16 / fp16 share the weights)
# and configs[3] (256x20b), at bench.py's seed
BENCHED = [("configs[1]/[4] 128x10b", 128, 9, 128), ("configs[3] 256x20b", 256, 19, 256)]


@pytest.mark.parametrize("name,C,R,hid", BENCHED)
def test_benched_nets_have_live_outputs(positions, name, C, R, hid):
    x, _ = positions
    sd = bench.bench_state_dict("live", 2025, 17, C, R, hid)
    p, v = _outputs(sd, x)
    assert v.std() >= 0.05, (name, v.std())
    assert abs(v.mean()) < 0.5
    ent = -(p * np.log(np.maximum(p, 1e-30))).sum(1).mean()
    assert ent < np.log(65) - 0.02, (name, ent)  # not uniform


def test_deep_tree_net_has_peaked_priors_and_a_live_value(positions):
    x, legal = positions
    sd = bench.bench_state_dict("frontier", 2025, 17, 128, 9, 128, sharpness=1.25)
    p, v = _outputs(sd, x)
    assert v.std() >= 0.05
    assert 0.3 <= p.max(1).mean() <= 0.5, p.max(1).mean()
    mass = (p * legal).sum(1)
    assert mass.mean() >= 0.6, mass.mean()  # most prior mass on legal moves, like a trained net


def test_selfplay_trained_net_is_trained_like(positions):
    """The deep_tree record's default net (bench_nets/, trained by
    tools/selfplay_train.py): priors on legal moves like a trained net's, a
    value spread over [-1, 1]."""
    x, legal = positions
    sd = bench.bench_state_dict("selfplay", 0, 17, 128, 9, 128)
    p, v = _outputs(sd, x)
    assert v.std() >= 0.3
    assert (p * legal).sum(1).mean() >= 0.95
    assert 0.3 <= p.max(1).mean() <= 0.5


def test_torch_default_init_is_degenerate(positions):
    """Why the bench moved off it: constant value, (near-)uniform priors."""
    x, _ = positions
    p, v = _outputs(bench.bench_state_dict("torch-default", 2025, 17, 128, 9, 128), x)
    assert v.std() < 1e-3
    assert -(p * np.log(p)).sum(1).mean() > np.log(65) - 0.02


def test_live_state_dict_is_deterministic_and_keyed_like_the_reference():
    from othello_mcts.synthetic import alphazero_state_dict, live_state_dict

    a = live_state_dict(3, 9, 128, 2, 32)
    b = live_state_dict(3, 9, 128, 2, 32)
    ref = alphazero_state_dict(3, 9, 128, 2, 32)
    assert list(a) == list(ref)
    assert all(a[k].shape == ref[k].shape and a[k].dtype == ref[k].dtype for k in a)
    assert all(np.array_equal(a[k], b[k]) for k in a)
    f = live_state_dict(3, 9, 128, 2, 32, policy="frontier")
    # the frontier channels pass every residual block unchanged (norm2 gamma = beta = 0)
    assert (f["residual_blocks.1.norm2.weight"][:2] == 0).all() and (f["residual_blocks.1.norm2.bias"][:2] == 0).all()
    with pytest.raises(ValueError):
        live_state_dict(3, 9, 128, 2, 32, policy="nope")


def test_fp16_headroom_of_the_drop_in_default():
    """The drop-in MCTS converts a module to fp16 only with FP16_HEADROOM (16x)
    below the fp16 maximum on real positions (othello_mcts.native, round 6):
    the trained and benched nets have thousands of x; a net whose activations
    would overflow fp16 has none and is evaluated in bf16."""
    from othello_mcts.native import FP16_HEADROOM, fp16_headroom
    from othello_mcts.synthetic import live_state_dict, selfplay_state_dict

    assert fp16_headroom(selfplay_state_dict(), 8) > 1000 * FP16_HEADROOM / 16
    live = live_state_dict(2025, 17, 128, 9, 128)
    assert fp16_headroom(live, 8) > 100
    blown = {k: (v * 300 if k.endswith("conv2.weight") else v) for k, v in live.items()}
    assert fp16_headroom(blown, 8) < FP16_HEADROOM

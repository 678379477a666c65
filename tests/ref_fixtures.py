"""Loader + replay for the reference-generated MCTS fixtures
(tests/golden/ref_mcts.*, ref_self_play.*; generator: tests/golden/make_ref_mcts.py,
which ran the compiled reference extension).

``replay_case`` drives any object with the reference's MCTS surface
(apply_action / search / visit_counts / mean_action_values / self_play_data /
position) through one case and compares every move bit for bit with what the
reference produced. It is shared by the oracle test (CPU) and the HIP test
(GPU), so both are held to the same reference record.
"""

from __future__ import annotations

import json
from pathlib import Path

import numpy as np

GOLD = Path(__file__).resolve().parent / "golden"


def real_features(n: int, history_size: int, seed: int) -> np.ndarray:
    """Feature planes of `n` real positions: seeded random games from the
    initial position (0-57 plies), each with its history and a random D4
    transform, built by the oracle restatement (pinned by the reference's
    feature vectors, test_oracle_golden.py). The ResNet goldens are the
    reference AlphaZeroNet's outputs on these planes (make_golden.py); the
    large ones store only (n, seed) and a checksum of the planes, which the
    tests regenerate here."""
    import oracle as O

    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        chain = [O.initial_position()]
        for _ in range(int(rng.integers(0, 58))):
            p = chain[-1]
            if p.player == 0:
                break
            acts = O.legal_actions(p)
            chain.append(O.apply_action(p, int(acts[rng.integers(len(acts))])))
        if chain[-1].player == 0:
            chain.pop()
        out.append(O.features(chain[::-1], history_size, int(rng.integers(8))))
    return np.stack(out).astype(np.float32)


def planes_checksum(x: np.ndarray) -> str:
    import hashlib

    return hashlib.sha256(np.ascontiguousarray(x.astype(np.int8)).tobytes()).hexdigest()[:16]


def weights_checksum(sd) -> str:
    import hashlib

    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(v).tobytes())
    return h.hexdigest()[:16]


def live_case(name: str):
    """(meta, state_dict, planes, golden) of a live-net golden
    (resnet_live.*, make_golden.py make_resnet_live): the weights regenerate
    from their seed (synthetic.live_state_dict) and the planes from theirs,
    both checked against the stored checksums."""
    from othello_mcts.synthetic import live_state_dict, selfplay_state_dict

    meta = json.loads((GOLD / "resnet_live_meta.json").read_text())[name]
    if meta["policy"] == "selfplay":
        sd = selfplay_state_dict()
    else:
        sd = live_state_dict(meta["seed"], 1 + 2 * meta["history_size"], meta["conv_channels"],
                             meta["num_residual_blocks"], meta["value_head_hidden_channels"], policy=meta["policy"],
                             policy_sharpness=meta["policy_sharpness"])
    assert weights_checksum(sd) == meta["weights_sha256_16"], "live_state_dict no longer reproduces the golden's weights"
    x = real_features(meta["boards"], meta["history_size"], meta["planes_seed"])
    assert planes_checksum(x) == meta["planes_sha256_16"]
    g = np.load(GOLD / "resnet_live.npz")
    return meta, sd, x, {"policy": g[f"{name}_policy"], "value": g[f"{name}_value"]}


LIVE_CASES = ["live_c128b9_h8_r1027", "frontier_c128b9_h8_r1027", "selfplay_c128b9_h8_r1027",
              "live_c256b19_h8_r1025"]


def load_cases() -> list[dict]:
    return json.loads((GOLD / "ref_mcts.json").read_text())["cases"]


_arrays = None


def arrays():
    global _arrays
    if _arrays is None:
        _arrays = dict(np.load(GOLD / "ref_mcts.npz"))
    return _arrays


def expected(case: dict) -> list[dict]:
    """Per-move expected records of a case."""
    a = arrays()
    name = case["name"]
    C = 1 + 2 * case["history_size"]
    offs = np.cumsum([0] + case["num_children"])
    visits, q = a[f"{name}__visits"], a[f"{name}__q_bits"].view(np.float32)
    feats = np.unpackbits(a[f"{name}__features_packed"], axis=2)[:, :, : C * 64]
    out = []
    for i, act in enumerate(case["actions"]):
        out.append({
            "root": case["root_positions"][i],
            "visits": visits[offs[i]:offs[i + 1]].tolist(),
            "q": q[offs[i]:offs[i + 1]],
            "features": feats[i].reshape(8, C, 8, 8).astype(np.float32),
            "policy": a[f"{name}__policy"][i],
            "action": act,
        })
    return out


def replay_case(m, case: dict, search, position_tuple, self_play_data) -> int:
    """Replay ``case`` on ``m``; returns the number of Q values that differ by
    more than 0 ulp but within 1e-6 (reported, not failed — SURVEY §4)."""
    for a in case["prefix"]:
        m.apply_action(a)
    ulp_flips = 0
    for i, exp in enumerate(expected(case)):
        assert position_tuple(m) == exp["root"], (case["name"], i, "root position")
        search(m)
        assert list(m.visit_counts()) == exp["visits"], (case["name"], i)
        q = np.array(m.mean_action_values(), np.float32)
        if not np.array_equal(q.view(np.uint32), exp["q"].view(np.uint32)):
            np.testing.assert_allclose(q, exp["q"], rtol=0, atol=1e-6, err_msg=f"{case['name']} move {i}")
            ulp_flips += int((q != exp["q"]).sum())
        f, p = self_play_data(m)
        np.testing.assert_array_equal(f, exp["features"], err_msg=f"{case['name']} move {i} features")
        np.testing.assert_array_equal(p, exp["policy"], err_msg=f"{case['name']} move {i} policy")
        m.apply_action(exp["action"])
    return ulp_flips


def load_self_play() -> tuple[list[dict], dict]:
    meta = json.loads((GOLD / "ref_self_play.json").read_text())
    return meta["games"], dict(np.load(GOLD / "ref_self_play.npz"))


def self_play_expected(games, arr, gi):
    g = games[gi]
    C = g["feature_shape"][0]
    n = g["samples"]
    f = np.unpackbits(arr[f"g{gi}__features_packed"], axis=1)[:, : C * 64].reshape(n, C, 8, 8)
    return f.astype(np.float32), arr[f"g{gi}__policy"], arr[f"g{gi}__values"]


def value_targets(num_moves: int, final_p1: int, final_p2: int) -> np.ndarray:
    """train.py:438-450's rule, restated: +-1/0 by final disc count for step 0,
    alternating sign per step, 8 samples per step."""
    b, w = bin(final_p1).count("1"), bin(final_p2).count("1")
    v = 1.0 if b > w else (-1.0 if b < w else 0.0)
    out = []
    for _ in range(num_moves):
        out += [v] * 8
        v = -v
    return np.array(out, np.float32)


def load_noise() -> tuple[list[dict], dict]:
    meta = json.loads((GOLD / "ref_noise.json").read_text())
    return meta["settings"], dict(np.load(GOLD / "ref_noise.npz"))


def compare_visit_distributions(ours: np.ndarray, ref: np.ndarray) -> tuple[float, float]:
    """Two-sample comparison of root visit counts (rows = independent runs,
    columns = root children): the smallest per-child KS p-value times the
    number of children (Bonferroni), and the largest std ratio deviation."""
    from scipy import stats

    assert ours.shape[1] == ref.shape[1]
    k = ours.shape[1]
    p = min(stats.ks_2samp(ours[:, j], ref[:, j]).pvalue for j in range(k)) * k
    ratio = max(abs(np.log(ours[:, j].std() / ref[:, j].std())) for j in range(k))
    return min(p, 1.0), float(np.exp(ratio))


# ---------------------------------------------------------------- racy endgames
def load_endgame_cases() -> list[dict]:
    """tests/golden/ref_mcts_endgame.json: T = 2 searches over a game's last
    plies, every distinct trajectory of 20 runs of the compiled reference."""
    return json.loads((GOLD / "ref_mcts_endgame.json").read_text())["cases"]


def endgame_trajectory(m, case: dict, search) -> tuple[list, list]:
    """Per-move visit counts and Q bit patterns of `m` over the case."""
    for a in case["prefix"]:
        m.apply_action(a)
    vis, qb = [], []
    for a in case["actions"]:
        search(m)
        vis.append([int(v) for v in m.visit_counts()])
        qb.append([int(x) for x in np.array(m.mean_action_values(), np.float32).view(np.uint32)])
        m.apply_action(a)
    return vis, qb


def matching_runs(case: dict, vis: list, qb: list) -> tuple[int, int]:
    """(runs, ulp flips): how many of the reference's runs followed this
    trajectory — every move's visit counts equal, Q within 1e-6 (SURVEY §4:
    the reference's own Q moves by an ulp with its random_device symmetry
    draws, which reorder the stub's float sums) — and how many Q values of the
    best-matching run differ in their bits. (0, _) = no reference run
    matches."""
    def close(t):
        if t["visits"] != vis:
            return None
        flips = 0
        for a, b in zip(t["q_bits"], qb):
            qa = np.array(a, np.uint32).view(np.float32)
            qo = np.array(b, np.uint32).view(np.float32)
            if np.abs(qa - qo).max(initial=0.0) > 1e-6:
                return None
            flips += int((qa != qo).sum())
        return flips
    hits = [(t["count"], f) for t in case["trajectories"] if (f := close(t)) is not None]
    if not hits:
        return 0, 0
    return sum(c for c, _ in hits), min(f for _, f in hits)

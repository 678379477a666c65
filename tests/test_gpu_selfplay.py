"""On-device self-play data path end to end on the GPU."""

import json

import pytest
import torch

import resnet_ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_self_play_samples_match_reference_format():
    import othello_mcts as om
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(4, 5, 128, 1, 32), device=0)
    b = om.BatchedMCTS(8, history_size=2, num_simulations=16, num_threads=1, batch_size=8, seed=3,
                       node_capacity=1 << 15)
    data = om.self_play(b, net, games=2)
    n = len(data["features"])
    assert n > 0 and n % 8 == 0 and len(data["policies"]) == n and len(data["values"]) == n
    for i in range(0, n, 8):
        vs = {float(v) for v in data["values"][i:i + 8]}
        assert len(vs) == 1 and vs <= {-1.0, 0.0, 1.0}
        f = data["features"][i]
        assert f.shape == (5, 8, 8) and f.device.type == "cpu"
        assert float(f[0].min()) == float(f[0].max())  # plane 0 constant
    pol = torch.stack(data["policies"])
    assert pol.shape == (n, 65)
    torch.testing.assert_close(pol.sum(1), torch.ones(n), atol=1e-5, rtol=0)
    # every game starts at the initial position: black to move, 4 discs
    f0 = data["features"][0]
    assert float(f0[0, 0, 0]) == 0.0 and int(f0[1].sum() + f0[2].sum()) == 4


def test_self_play_multi_move_calls_equal_move_by_move():
    """self_play with a native net runs selfplay_steps chunks (free-running
    games); every game's moves are those of the move-by-move loop, so the
    samples of the games the move-by-move run completed come out first and
    identical."""
    import othello_mcts as om
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(4, 5, 128, 1, 32), device=0)

    def run(chunk):
        b = om.BatchedMCTS(16, history_size=2, num_simulations=32, num_threads=2, batch_size=8, seed=5,
                           node_capacity=1 << 15)
        b.random_openings(40, seed=9)  # late openings: games complete within a few moves
        return om.self_play(b, net, games=6, opening_moves=4, moves_per_call=chunk)

    a, c = run(1), run(8)
    n = len(a["features"])
    assert n > 0 and len(c["features"]) >= n
    for k in ("features", "policies", "values"):
        assert all(torch.equal(x, y) for x, y in zip(a[k], c[k][:n])), k


def test_native_net_from_reference_checkpoint(tmp_path):
    import othello_mcts as om
    from othello_mcts.synthetic import alphazero_state_dict, net_config_from_state_dict

    sd = {k: torch.from_numpy(v) for k, v in alphazero_state_dict(6, 17, 128, 3, 64).items()}
    torch.save(sd, tmp_path / "neural_net.pth")
    (tmp_path / "config.json").write_text(json.dumps({"neural_net": net_config_from_state_dict(sd)}))
    net = om.NativeNet.from_checkpoint(tmp_path, device=0)
    x = (torch.rand((64, 17, 8, 8), generator=torch.Generator().manual_seed(1)) < 0.3).float().to(DEV)
    ref = resnet_ref.forward(sd, x)
    out = net(x)
    assert (out["policy"] - ref["policy"]).abs().max().item() <= 2e-3
    assert (out["value"] - ref["value"]).abs().max().item() <= 1e-2


# ------------------------------------------------------------------------------
# On-device self-play driver vs the oracle (train.py:404-452,
# mcts.cpp:63-112)
# ------------------------------------------------------------------------------
import numpy as np  # noqa: E402

import numerics  # noqa: E402
import oracle as O  # noqa: E402


def _stub(features):
    p, v = O.equivariant_stub(features.cpu().numpy())
    return {"policy": torch.from_numpy(p), "value": torch.from_numpy(v)}


def test_selfplay_driver_targets_and_moves_match_oracle():
    """k_selfplay_move, move by move for every game: its 8-fold features and
    policies equal the oracle's self_play_data bit for bit, and the action it
    plays is the oracle's restatement of train.py:421-430 drawn from the same
    random event (temperature sampling for 12 plies, then argmax with random
    tie-break). Dirichlet noise on, so every game differs."""
    import othello_mcts as om

    G, H, moves = 16, 4, 18
    kw = dict(history_size=H, num_simulations=64, num_threads=2, batch_size=8, dirichlet_epsilon=0.25)
    b = om.BatchedMCTS(G, seed=41, node_capacity=1 << 16, **kw)
    refs = [O.OracleMCTS(game_key=b.engine.game_key(g), **kw) for g in range(G)]
    for ply in range(moves):
        b.search(_stub)
        for r in refs:
            r.search(O.equivariant_stub)
        out = b.selfplay_move(temperature_moves=12, temperature=1.0, opening_moves=0, emit_targets=True)
        acts = out["actions"].cpu().numpy()
        fin = out["finished"].cpu().numpy()
        feats = out["features"].cpu().numpy()
        pols = out["policy"].cpu().numpy()
        for g, r in enumerate(refs):
            f, p = r.self_play_data()
            np.testing.assert_array_equal(feats[g], f, err_msg=f"ply {ply} game {g} features")
            np.testing.assert_array_equal(pols[g], p, err_msg=f"ply {ply} game {g} policy")
            vc = np.array(r.visit_counts())
            a = r.selfplay_action(ply, 12, 1.0)
            assert acts[g] == a, (ply, g, acts[g], a, vc)
            k = O.legal_actions(r.position()).index(a)
            assert vc[k] > 0 if ply < 12 else vc[k] == vc.max()
            assert fin[g] == 0  # 18 plies from the initial position: no game ends
            r.apply_action(a)


def _tied_roots(om, G, seed):
    """G games at the initial position searched with the uniform stub and
    T=1, eps=0: every root has 4 children at 76 visits (reference known answer
    uni_h8_b16_s320_open, tests/golden/ref_mcts.json)."""
    b = om.BatchedMCTS(G, history_size=8, num_simulations=320, num_threads=1, batch_size=16,
                       dirichlet_epsilon=0.0, seed=seed, node_capacity=1 << 14)

    def uni(features):
        p, v = O.uniform_stub(features.cpu().numpy())
        return {"policy": torch.from_numpy(p), "value": torch.from_numpy(v)}

    b.search(uni)
    v, _ = b.root_stats()
    v = v.cpu().numpy()
    assert (v[:, [19, 26, 37, 44]] == 76).all() and v.sum() == 4 * 76 * G
    return b


def test_selfplay_argmax_tie_break_is_uniform():
    """train.py:428-430: argmax with np.random.choice over the tied indices.
    Constructed 4-way ties on every root; the driver's picks over 4 x 512
    games must be uniform (chi-square, 3 dof, p > 0.001)."""
    import othello_mcts as om

    counts = {19: 0, 26: 0, 37: 0, 44: 0}
    for seed in range(4):
        b = _tied_roots(om, 512, 100 + seed)
        acts = b.selfplay_move(temperature_moves=0)["actions"].cpu().numpy()  # argmax from ply 0
        for a in acts:
            counts[int(a)] += 1
    n = sum(counts.values())
    exp = n / 4
    chi2 = sum((c - exp) ** 2 / exp for c in counts.values())
    numerics.record("selfplay tie-break", f"counts={counts} chi2={chi2:.2f} (3 dof, p=0.001 at 16.27)")
    assert n == 2048 and chi2 < 16.27


@pytest.mark.parametrize("temperature", [1.0, 0.5])
def test_selfplay_temperature_sampling_follows_visit_powers(temperature):
    """train.py:421-426: p ~ N^(1/tau). Heterogeneous roots (random openings,
    equivariant stub); every draw's randomized probability-integral transform
    under p must be Uniform(0, 1): chi-square over 10 bins, >= 10k draws."""
    import othello_mcts as om

    rng = np.random.default_rng(5)
    pit = []
    for rep in range(5):
        b = om.BatchedMCTS(2048, history_size=4, num_simulations=32, num_threads=1, batch_size=16,
                           dirichlet_epsilon=0.0, seed=300 + rep, node_capacity=1 << 12)
        b.random_openings(10, seed=rep)
        b.search(_stub)
        v, _ = b.root_stats()
        v = v.cpu().numpy().astype(np.float64)
        acts = b.selfplay_move(temperature_moves=12, temperature=temperature)["actions"].cpu().numpy()
        w = v ** (1.0 / temperature)
        for g in range(v.shape[0]):
            if w[g].sum() == 0:
                continue
            p = w[g] / w[g].sum()
            a = int(acts[g])
            assert p[a] > 0, (g, a)
            pit.append(p[:a].sum() + rng.random() * p[a])
    pit = np.array(pit)
    hist, _ = np.histogram(pit, bins=10, range=(0.0, 1.0))
    exp = len(pit) / 10
    chi2 = float(((hist - exp) ** 2 / exp).sum())
    numerics.record(f"selfplay sampling tau={temperature}", f"draws={len(pit)} chi2={chi2:.2f} (9 dof, p=0.001 at 27.88)")
    assert len(pit) >= 10000 and chi2 < 27.88


# ------------------------------------------------------------------------------
# Node-pool exhaustion is an error, never a silent divergence
# ------------------------------------------------------------------------------
def test_node_pool_overflow_raises():
    import othello_mcts as om

    m = om.MCTS(history_size=4, torch_device="cuda:0", num_simulations=800, num_threads=1, batch_size=16,
                dirichlet_epsilon=0.0, node_capacity=256, seed=1)
    m.set_native_nn(False)
    with pytest.raises(RuntimeError, match="node pool exhausted"):
        m.search(_stub)
    b = om.BatchedMCTS(4, history_size=4, num_simulations=800, num_threads=1, batch_size=16, seed=2,
                       node_capacity=512)
    with pytest.raises(RuntimeError, match="node pool exhausted"):
        b.search(_stub)
    # the asynchronous native search is caught by the collector
    from othello_mcts.selfplay import SelfPlayCollector
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(4, 9, 128, 1, 32), device=0)
    b = om.BatchedMCTS(4, history_size=4, num_simulations=800, num_threads=1, batch_size=16, seed=2,
                       node_capacity=512)
    b.search(net, sync=False)
    col = SelfPlayCollector(4)
    with pytest.raises(RuntimeError, match="node pool exhausted"):
        col.add(b.selfplay_move(emit_targets=True))


def test_collector_rejects_unexpanded_roots():
    """selfplay_move without a search first: no targets exist; the collector
    raises the reference's self_play_data message (mcts.cpp:69-71)."""
    import othello_mcts as om
    from othello_mcts.selfplay import FIN_NO_TARGETS, SelfPlayCollector

    b = om.BatchedMCTS(4, history_size=4, num_simulations=32, num_threads=1, batch_size=8, seed=2,
                       node_capacity=1 << 12)
    out = b.selfplay_move(emit_targets=True)
    assert ((out["finished"].cpu() & FIN_NO_TARGETS) != 0).all()
    with pytest.raises(ValueError, match="The root node has not been expanded yet."):
        SelfPlayCollector(4).add(out)


def test_device_sample_buffer_training_and_refresh():
    """self-play samples stay in HBM (SampleBuffer == the host
    collector's samples), a training epoch runs on them on the device, and the
    trained weights reach the engine's NativeNet (refresh_native == a fresh
    NativeNet of those weights, bit for bit)."""
    import othello_mcts as om
    from othello_mcts.selfplay import SelfPlayCollector
    from othello_mcts.synthetic import alphazero_state_dict
    from othello_mcts.training import SampleBuffer, refresh_native, train_epoch

    G = 16
    net = om.NativeNet(alphazero_state_dict(4, 5, 128, 1, 32), device=0)
    b = om.BatchedMCTS(G, history_size=2, num_simulations=16, num_threads=1, batch_size=8, seed=3,
                       node_capacity=1 << 14)
    col = SelfPlayCollector(G, device=DEV)
    buf = SampleBuffer(G, 5, capacity=1 << 14, device=DEV)
    ref = {"features": [], "policies": [], "values": []}
    while col.games_completed < G:
        b.search(net)
        out = b.selfplay_move(emit_targets=True)
        buf.add(out)
        got = col.add(out)
        for k in ref:
            ref[k] += got[k]
    assert buf.games_completed == col.games_completed and buf.size == len(ref["values"])
    assert torch.equal(buf.features[:buf.size], torch.stack(ref["features"]))
    assert torch.equal(buf.policies[:buf.size], torch.stack(ref["policies"]))
    assert torch.equal(buf.values[:buf.size], torch.stack(ref["values"]))

    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = torch.nn.Linear(5 * 64, 66)

        def forward(self, x):
            y = self.lin(x.flatten(1))
            return {"policy": torch.softmax(y[:, :65], 1), "value": torch.tanh(y[:, 65])}

    toy = Toy().to(DEV)
    opt = torch.optim.SGD(toy.parameters(), lr=0.1, momentum=0.9)
    means = train_epoch(toy, opt, buf.features[:buf.size], buf.policies[:buf.size], buf.values[:buf.size],
                        batch_size=64)
    assert all(np.isfinite(v) for v in means.values()) and means["policy_loss"] > 0

    sd2 = alphazero_state_dict(9, 5, 128, 1, 32)

    class Holder(torch.nn.Module):  # stands in for the trained AlphaZeroNet
        def state_dict(self, *a, **k):
            return {k_: torch.from_numpy(np.asarray(v)) for k_, v in sd2.items()}

    refresh_native(net, Holder())
    fresh = om.NativeNet(sd2, device=0)
    x = buf.features[:300].contiguous()
    o1, o2 = net(x), fresh(x)
    assert torch.equal(o1["policy"], o2["policy"]) and torch.equal(o1["value"], o2["value"])

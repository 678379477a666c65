"""GPU parity tests (run on an MI355X with ``-m gpu``): HIP kernels through the
C ABI vs the oracle and the reference's golden vectors.

Bars (DESIGN.md "Parity"):
  * bitboards, transforms, features, tree statistics: bit-exact;
  * MCTS visit counts / mean action values with an external evaluator: bit-exact
    vs the oracle (same random stream spec), incl. Dirichlet noise, T > 1 and
    tree reuse; known-answer visit counts of the reference;
  * native ResNet (bf16 / fp16 MFMA, fp32 accumulate): see test_gpu_resnet.py.
"""

import json
import time

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def u64(a):
    return np.asarray(a).view(np.uint64)


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a).view(np.int64))).to(DEV)


@pytest.fixture(scope="module")
def om():
    import othello_mcts

    assert othello_mcts.device_count() >= 1
    return othello_mcts


@pytest.fixture(scope="module")
def bb(golden_dir):
    d = np.load(golden_dir / "bitboards.npz")
    return {k: d[k] for k in d.files}


def _impl(om):
    return om._othello_mcts_impl


def gpu_legal(om, me, opp):
    me_t, opp_t = to_dev(me), to_dev(opp)
    out = torch.empty_like(me_t)
    s = torch.cuda.current_stream().cuda_stream
    _impl(om)._gpu_legal_moves(me_t.data_ptr(), opp_t.data_ptr(), out.data_ptr(), me_t.numel(), s)
    return out.cpu().numpy().view(np.uint64)


def gpu_flips(om, mv, me, opp):
    mv_t, me_t, opp_t = to_dev(mv), to_dev(me), to_dev(opp)
    out = torch.empty_like(me_t)
    s = torch.cuda.current_stream().cuda_stream
    _impl(om)._gpu_flips(mv_t.data_ptr(), me_t.data_ptr(), opp_t.data_ptr(), out.data_ptr(), me_t.numel(), s)
    return out.cpu().numpy().view(np.uint64)


def pack_positions(player, p1, p2, legal, nxt):
    n = len(player)
    rec = np.zeros((n, 5), np.uint64)
    rec[:, 0] = np.asarray(player, np.int64).astype(np.uint64)  # int32 player + int32 reserved
    rec[:, 1], rec[:, 2], rec[:, 3], rec[:, 4] = u64(p1), u64(p2), u64(legal), u64(nxt)
    return rec


def gpu_apply(om, rec, actions):
    rin = torch.from_numpy(rec.view(np.int64)).to(DEV)
    act = torch.from_numpy(np.asarray(actions, np.int32)).to(DEV)
    out = torch.empty_like(rin)
    s = torch.cuda.current_stream().cuda_stream
    _impl(om)._gpu_apply_action(rin.data_ptr(), act.data_ptr(), out.data_ptr(), len(rec), s)
    o = out.cpu().numpy().view(np.uint64)
    return (o[:, 0] & 0xFFFFFFFF).astype(np.int32), o[:, 1], o[:, 2], o[:, 3], o[:, 4]


# --------------------------------------------------------------------- bitboards
def test_gpu_legal_moves_golden(om, bb):
    got = gpu_legal(om, bb["rnd_me"], bb["rnd_opp"])
    np.testing.assert_array_equal(got, u64(bb["rnd_legal"]))
    pl, p1, p2 = bb["pos_player"], u64(bb["pos_p1"]), u64(bb["pos_p2"])
    idx = bb["lm_index"]
    me = np.where(pl[idx] == 1, p1[idx], p2[idx])
    opp = np.where(pl[idx] == 1, p2[idx], p1[idx])
    np.testing.assert_array_equal(gpu_legal(om, me, opp), u64(bb["lm_value"]))


def test_gpu_flips_golden(om, bb):
    i = bb["fl_index"]
    mv = (np.uint64(1) << (np.uint64(63) - bb["fl_square"].astype(np.uint64)))
    got = gpu_flips(om, mv, u64(bb["rnd_me"])[i], u64(bb["rnd_opp"])[i])
    np.testing.assert_array_equal(got, u64(bb["fl_flips"]))


def test_gpu_apply_action_golden(om, bb):
    par, a = bb["ch_parent"], bb["ch_action"]
    pl, p1, p2, lg = bb["pos_player"][par], u64(bb["pos_p1"])[par], u64(bb["pos_p2"])[par], u64(bb["pos_legal"])[par]
    me = np.where(pl == 1, p1, p2)
    opp = np.where(pl == 1, p2, p1)
    nxt = np.where(lg == 0, O.legal_moves_n(opp, me), np.uint64(0))  # position.h:351-357
    player, c1, c2, cl, _ = gpu_apply(om, pack_positions(pl, p1, p2, lg, nxt), a)
    np.testing.assert_array_equal(player, bb["ch_player"])
    np.testing.assert_array_equal(c1, u64(bb["ch_p1"]))
    np.testing.assert_array_equal(c2, u64(bb["ch_p2"]))
    np.testing.assert_array_equal(cl, u64(bb["ch_legal"]))


def test_gpu_bitboards_large_random_vs_oracle(om):
    """Full-size batch (4M boards) against the C oracle, bit-exact."""
    rng = np.random.default_rng(5)
    n = 1 << 22
    occ = rng.integers(0, 2**63, n, dtype=np.uint64) | rng.integers(0, 2**63, n, dtype=np.uint64) << np.uint64(1)
    occ &= rng.integers(0, 2**63, n, dtype=np.uint64) << np.uint64(1) | rng.integers(0, 2**63, n, dtype=np.uint64)
    split = rng.integers(0, 2**63, n, dtype=np.uint64) << np.uint64(1)
    me, opp = occ & split, occ & ~split
    np.testing.assert_array_equal(gpu_legal(om, me, opp), O.legal_moves_n(me, opp))
    mv = np.uint64(1) << rng.integers(0, 64, n).astype(np.uint64)
    np.testing.assert_array_equal(gpu_flips(om, mv, me, opp), O.flips_n(mv, me, opp))


def test_gpu_apply_action_random_games_vs_oracle(om):
    """Play 2048 random games in lock-step on the GPU, checking every ply."""
    rng = np.random.default_rng(9)
    n = 2048
    ip = O.initial_position()
    player = np.full(n, 1, np.int32)
    p1 = np.full(n, ip.p1, np.uint64)
    p2 = np.full(n, ip.p2, np.uint64)
    lg = np.full(n, ip.legal, np.uint64)
    nx = np.zeros(n, np.uint64)
    for _ in range(70):
        act = np.zeros(n, np.int32)
        for i in range(n):
            if player[i] == 0:
                act[i] = 64  # terminal: pass keeps the board (value ignored below)
                continue
            if lg[i] == 0:
                act[i] = 64
            else:
                bits = [s for s in range(64) if (int(lg[i]) >> (63 - s)) & 1]
                act[i] = bits[rng.integers(len(bits))]
        live = player != 0
        g = gpu_apply(om, pack_positions(player, p1, p2, lg, nx), act)
        o = O.apply_action_n(player, p1, p2, lg, nx, act)
        for x, y in zip(g, o):
            np.testing.assert_array_equal(x[live], y[live])
        player = np.where(live, g[0], player)
        p1, p2, lg, nx = (np.where(live, x, y) for x, y in zip(g[1:], (p1, p2, lg, nx)))
        if not live.any():
            break


# --------------------------------------------------------------------- MCTS
def _mcts(om, **kw):
    base = dict(history_size=4, torch_device="cpu", num_simulations=800, num_threads=1, batch_size=16,
                dirichlet_epsilon=0.0, seed=1234)
    base.update(kw)
    m = om.MCTS(**base)
    m.set_native_nn(False)
    return m


def _torch_stub(fn):
    def nn(features):
        p, v = fn(features.cpu().numpy())
        return {"policy": torch.from_numpy(p), "value": torch.from_numpy(v)}
    return nn


@pytest.mark.parametrize("case", json.load(open(__import__("pathlib").Path(__file__).parent / "golden"
                                               / "mcts_known_answers.json"))["cases"], ids=lambda c: c["name"])
def test_gpu_mcts_known_answers(om, case):
    m = _mcts(om, history_size=case["history_size"], num_simulations=case["num_simulations"],
              num_threads=case["num_threads"], batch_size=case["batch_size"],
              dirichlet_epsilon=case["dirichlet_epsilon"])
    for a in case["actions"]:
        m.apply_action(a)
    stub = O.equivariant_stub if case["stub"] == "equivariant" else O.uniform_stub
    m.search(_torch_stub(stub))
    assert m.visit_counts() == case["visit_counts"]


import numerics  # noqa: E402
import ref_fixtures as RF  # noqa: E402

REF_ULP_FLIPS: dict[str, int] = {}


def _om_pos(m):
    p = m.position()
    return [int(p.player()), f"{p.player1_discs():016x}", f"{p.player2_discs():016x}", f"{p.legal_moves():016x}"]


def _om_spd(m):
    d = m.self_play_data()
    return torch.stack(d["features"]).numpy(), torch.stack(d["policy"]).numpy()


@pytest.mark.parametrize("case", RF.load_cases(), ids=lambda c: c["name"])
def test_gpu_mcts_matches_reference_matrix(om, case):
    """HIP search vs the COMPILED REFERENCE (tests/golden/make_ref_mcts.py):
    every move's visit counts, Q bits, 8-fold features and policies, with tree
    reuse over the case's fixed action sequence (search_thread.cpp:59-260,
    mcts.cpp:45-165). Q is allowed 1e-6; ulp flips are reported."""
    m = _mcts(om, history_size=case["history_size"], num_simulations=case["num_simulations"],
              num_threads=case["num_threads"], batch_size=case["batch_size"], dirichlet_epsilon=0.0)
    stub = _torch_stub(O.equivariant_stub if case["stub"] == "equivariant" else O.uniform_stub)
    flips = RF.replay_case(m, case, lambda mm: mm.search(stub), _om_pos, _om_spd)
    REF_ULP_FLIPS[case["name"]] = flips
    numerics.record(f"reference MCTS {case['name']}", f"moves={len(case['actions'])} q_ulp_flips={flips}")


def _endgame_ids():
    try:
        return RF.load_endgame_cases()
    except FileNotFoundError:  # pragma: no cover
        return []


@pytest.mark.parametrize("case", _endgame_ids(), ids=lambda c: c["name"])
def test_gpu_endgame_races_reproduce_a_reference_run(om, case):
    """The HIP search (drop-in MCTS, T = 2, k_tree's per-thread batch state) over
    the last plies of a game, where whole batches are terminal and the
    reference races (tests/golden/ref_mcts_endgame.json: 15-19 distinct
    trajectories in 20 runs): its trajectory must be one the reference
    produced, every move's visits exactly and Q within 1e-6
    (search_thread.cpp:47-128)."""
    m = _mcts(om, history_size=case["history_size"], num_simulations=case["num_simulations"],
              num_threads=case["num_threads"], batch_size=case["batch_size"], dirichlet_epsilon=0.0)
    stub = _torch_stub(O.equivariant_stub if case["stub"] == "equivariant" else O.uniform_stub)
    vis, qb = RF.endgame_trajectory(m, case, lambda mm: mm.search(stub))
    runs, flips = RF.matching_runs(case, vis, qb)
    numerics.record(f"reference endgame race {case['name']}",
                    f"follows a trajectory {runs} of {case['repeats']} reference runs took "
                    f"({len(case['trajectories'])} distinct), q_ulp_flips={flips}")
    assert runs > 0


@pytest.mark.parametrize("gi", [0, 1])
def test_gpu_reproduces_reference_self_play(om, gi):
    """The reference's train._self_play game (compiled reference MCTS, np.random
    seeded) replayed through the HIP MCTS drop-in: same per-move 8-fold targets,
    every chosen action admitted by train.py:421-430's rule, same value targets
    (train.py:438-450) from othello_mcts.selfplay's outcome rule."""
    from othello_mcts.selfplay import value_targets_from_outcome

    games, arr = RF.load_self_play()
    g = games[gi]
    f_exp, p_exp, v_exp = RF.self_play_expected(games, arr, gi)
    prm = g["params"]
    m = _mcts(om, history_size=prm["history_size"], num_simulations=prm["num_simulations"],
              num_threads=prm["num_threads"], batch_size=prm["batch_size"],
              dirichlet_epsilon=prm["dirichlet_epsilon"])
    stub = _torch_stub(O.equivariant_stub)
    black_to_move = []
    for t, a in enumerate(g["actions"]):
        pos = m.position()
        black_to_move.append(pos.player() == 1)
        m.search(stub)
        vc = np.array(m.visit_counts())
        k = pos.legal_actions().index(a)
        assert vc[k] > 0 if t < g["temperature_moves"] else vc[k] == vc.max()
        f, p = _om_spd(m)
        np.testing.assert_array_equal(f, f_exp[8 * t: 8 * t + 8])
        np.testing.assert_array_equal(p, p_exp[8 * t: 8 * t + 8])
        m.apply_action(a)
    fin = m.position()
    assert fin.is_terminal()
    v = value_targets_from_outcome(black_to_move, fin.player1_discs(), fin.player2_discs())
    np.testing.assert_array_equal(np.repeat(np.array(v, np.float32), 8), v_exp)


def _play_vs_oracle(om, moves, **kw):
    m = _mcts(om, **kw)
    ref = O.OracleMCTS(history_size=kw.get("history_size", 4), num_simulations=kw.get("num_simulations", 800),
                       num_threads=kw.get("num_threads", 1), batch_size=kw.get("batch_size", 16),
                       dirichlet_epsilon=kw.get("dirichlet_epsilon", 0.0),
                       dirichlet_alpha=kw.get("dirichlet_alpha", 0.5), game_key=m.game_key())
    stub = _torch_stub(O.equivariant_stub)
    for mv in range(moves):
        if m.position().is_terminal():
            break
        m.search(stub)
        ref.search(O.equivariant_stub)
        vc = m.visit_counts()
        assert vc == ref.visit_counts(), f"move {mv}"
        q = np.array(m.mean_action_values(), np.float32)
        np.testing.assert_array_equal(q, np.array(ref.mean_action_values(), np.float32))
        d = m.self_play_data()
        f, p = ref.self_play_data()
        np.testing.assert_array_equal(torch.stack(d["features"]).numpy(), f)
        np.testing.assert_array_equal(torch.stack(d["policy"]).numpy(), p)
        legal = m.position().legal_actions()
        a = legal[int(np.argmax(vc))]
        m.apply_action(a)
        ref.apply_action(a)


def test_gpu_mcts_matches_oracle_single_thread(om):
    _play_vs_oracle(om, 6, history_size=4, num_threads=1, batch_size=16)


def test_gpu_mcts_matches_oracle_two_threads_noise(om):
    # self-play defaults: T=2 x B=16, eps=0.25, alpha=0.5, H=8
    _play_vs_oracle(om, 6, history_size=8, num_threads=2, batch_size=16, dirichlet_epsilon=0.25)


def test_gpu_mcts_matches_oracle_many_leaves_per_step(om):
    # L = 3 x 48 = 144 leaves per step: k_backup's per-chunk prefetch runs over
    # chunks of 64, 64 and 16 leaves; duplicates within a step are frequent
    _play_vs_oracle(om, 4, history_size=8, num_threads=3, batch_size=48, dirichlet_epsilon=0.25)


def test_gpu_mcts_matches_oracle_max_history(om):
    # history_size = 15: 31 input planes, the widest packed feature row
    _play_vs_oracle(om, 3, history_size=15, num_simulations=256, num_threads=2, batch_size=16,
                    dirichlet_epsilon=0.25)


def test_gpu_mcts_matches_oracle_max_leaves_per_step(om):
    # num_threads * batch_size = 1024 (the engine's limit): one step per search,
    # 16 backup chunks of 64 leaves, most leaves duplicates of few nodes
    _play_vs_oracle(om, 2, history_size=4, num_simulations=1024, num_threads=4, batch_size=256)


def test_gpu_mcts_matches_oracle_endgame_passes(om):
    """Deep into random games (terminal leaves, passes, tree reuse over many moves)."""
    m = _mcts(om, history_size=3, num_simulations=96, num_threads=2, batch_size=8, dirichlet_epsilon=0.25)
    ref = O.OracleMCTS(history_size=3, num_simulations=96, num_threads=2, batch_size=8,
                       dirichlet_epsilon=0.25, game_key=m.game_key())
    stub = _torch_stub(O.equivariant_stub)
    moves = 0
    while not m.position().is_terminal():
        m.search(stub)
        ref.search(O.equivariant_stub)
        vc = m.visit_counts()
        assert vc == ref.visit_counts(), f"move {moves}"
        np.testing.assert_array_equal(np.array(m.mean_action_values(), np.float32),
                                      np.array(ref.mean_action_values(), np.float32))
        a = m.position().legal_actions()[int(np.argmax(vc))]
        m.apply_action(a)
        ref.apply_action(a)
        moves += 1
    assert moves >= 30
    assert ref.position().player == 0


def test_gpu_mcts_errors_match_reference(om, golden_dir):
    m = _mcts(om)
    with pytest.raises(IndexError, match=r"Expected 0 <= action < 65, but got 65\."):
        m.apply_action(65)
    with pytest.raises(ValueError, match=r"^0 is not a legal action\.$"):
        m.apply_action(0)
    with pytest.raises(ValueError, match="Pass is not allowed when there are legal moves."):
        m.apply_action(64)
    with pytest.raises(ValueError, match="The root node has not been expanded yet."):
        m.self_play_data()
    with pytest.raises(ValueError, match=r"Expected batch_size >= 1, but got 0\."):
        m.set_batch_size(0)
    with pytest.raises(ValueError, match=r"Expected c_puct_base > 0\.0, but got 0\.000000\."):
        m.set_c_puct_base(0.0)
    assert m.batch_size() == 16


def test_gpu_batched_games_match_single_game_oracle(om):
    """G games in one engine: each game equals its own single-game oracle."""
    G = 6
    b = om.BatchedMCTS(G, history_size=4, num_simulations=64, num_threads=2, batch_size=8,
                       dirichlet_epsilon=0.25, seed=77, node_capacity=1 << 16)

    def stub(features):
        p, v = O.equivariant_stub(features.cpu().numpy())
        return {"policy": torch.from_numpy(p), "value": torch.from_numpy(v)}

    refs = [O.OracleMCTS(history_size=4, num_simulations=64, num_threads=2, batch_size=8,
                         dirichlet_epsilon=0.25, game_key=b.engine.game_key(g)) for g in range(G)]
    for mv in range(4):
        b.search(stub)
        acts = torch.full((G,), -1, dtype=torch.int32)
        for g, r in enumerate(refs):
            r.search(O.equivariant_stub)
            assert b.visit_counts(g) == r.visit_counts(), (mv, g)
            vc = r.visit_counts()
            a = O.legal_actions(r.position())[int(np.argmax(vc))]
            acts[g] = a
            r.apply_action(a)
        b.apply_actions(acts.to(DEV))


def test_gpu_selfplay_driver(om):
    G = 32
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(5, 9, 128, 2, 32), device=0)
    b = om.BatchedMCTS(G, history_size=4, num_simulations=64, num_threads=2, batch_size=16, seed=3,
                       node_capacity=1 << 16)
    b.random_openings(8, seed=11)
    finished = 0
    for mv in range(70):
        sims, evals = b.search(net)
        assert sims == G * 64
        assert 0 < evals <= sims
        out = b.selfplay_move(temperature_moves=12, opening_moves=4, emit_targets=True)
        acts = out["actions"].cpu().numpy()
        assert (acts >= 0).all() and (acts <= 64).all()
        pol = out["policy"].cpu().numpy()
        np.testing.assert_allclose(pol.sum(-1), 1.0, atol=1e-5)
        feat = out["features"].cpu().numpy()
        assert set(np.unique(feat)) <= {0.0, 1.0}
        finished += int((out["finished"].cpu().numpy() > 0).sum())
    assert finished >= G // 2  # 70 plies: most games ended and restarted
    for g in range(G):
        info = b.root_info(g)
        assert info["overflow"] == 0


def test_gpu_async_search_matches_sync(om):
    """search(sync=False) only enqueues; a loop of async searches + on-device
    moves gives the same games as the synchronous loop, and the lazily summed
    HIP-event timing counts every launch."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(5, 9, 128, 2, 32), device=0)
    G, moves = 96, 6

    def play(sync):
        b = om.BatchedMCTS(G, history_size=4, num_simulations=64, num_threads=2, batch_size=16, seed=9,
                           node_capacity=1 << 17)
        b.random_openings(6, seed=4)
        b.engine.set_chain_split(1, 3)  # up to 3 extra rounds per search (chain splitting)
        b.engine.enable_timing(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        acts = []
        for _ in range(moves):
            r = b.search(net, sync=sync)
            assert (r is None) == (not sync)
            acts.append(b.selfplay_move(temperature_moves=3, emit_targets=False)["actions"].clone())
        ms, launches, rows = b.engine.nn_timing()
        sel, bk, launches2 = b.engine.tree_timing()
        # every round is timed, the extra chain-splitting rounds included: 2
        # batches per thread + X in [1, 3] per search (adaptive: the first two
        # searches run the minimum, 1)
        searches, rounds, finals = b.engine.round_counts()
        assert searches == moves and moves * 3 <= rounds <= moves * 5
        assert launches2 == rounds * 2 and finals == moves * 2  # 2 pipeline groups at G >= 64
        timed_groups = 2  # every group's NN launches carry events
        assert launches == rounds * timed_groups
        assert rows == rounds * (G // 2) * 32 * timed_groups
        assert ms > 0 and sel > 0 and bk > 0
        # busy: the union of the kernel-recorded intervals of every ResNet
        # launch since enable_timing, at most the event spans' sum (two NN
        # chains by default, so the groups' launches may overlap)
        busy, busy_launches = b.engine.nn_busy()
        wall_ms = (time.perf_counter() - t0) * 1e3
        assert 0 < busy <= ms * 1.0001 and busy <= wall_ms  # a union of the window's launches
        assert busy_launches == launches  # every search timed here: the same launches
        return torch.stack(acts).cpu().numpy(), [b.visit_counts(g) for g in range(G)]

    a_sync, v_sync = play(True)
    a_async, v_async = play(False)
    np.testing.assert_array_equal(a_sync, a_async)
    assert v_sync == v_async


@pytest.mark.parametrize("idx", [0, 1, 2])
def test_gpu_dirichlet_noise_distribution_matches_reference(om, idx):
    """The HIP search's root visit counts under Dirichlet noise over independent
    games vs the compiled reference's over as many runs (tests/golden/ref_noise.*):
    per-child two-sample KS (Bonferroni p > 1e-3), per-child std within 25 %.
    Setting 2 is the self-play configuration's thread structure (T=2 x B=16,
    800 sims, H=8)."""
    settings, arr = RF.load_noise()
    st = settings[idx]
    G = st["runs"]
    b = om.BatchedMCTS(G, history_size=st["history_size"], num_simulations=st["num_simulations"],
                       num_threads=st["num_threads"], batch_size=st["batch_size"], dirichlet_epsilon=0.25,
                       dirichlet_alpha=0.5, seed=91 + idx, node_capacity=1 << 15)
    for a in st["prefix"]:
        b.apply_actions(torch.full((G,), a, dtype=torch.int32, device=DEV))

    def stub(features):
        p, v = O.equivariant_stub(features.cpu().numpy())
        return {"policy": torch.from_numpy(p), "value": torch.from_numpy(v)}

    b.search(stub)
    v, _ = b.root_stats()
    ours = v[:, _legal_of(b)].cpu().numpy()
    p, r = RF.compare_visit_distributions(ours, arr[st["name"]])
    numerics.record(f"dirichlet noise {st['name']}", f"games={G} ks_bonferroni_p={p:.3g} max_std_ratio={r:.3f}")
    assert p > 1e-3 and r < 1.25, (st["name"], p, r)


def _legal_of(b):
    """Root children's actions of game 0 (legal_actions order)."""
    info = b.root_info(0)
    legal = info["legal_moves"]
    return [a for a in range(64) if (legal >> (63 - a)) & 1] or [64]

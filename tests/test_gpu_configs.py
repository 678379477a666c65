"""The single-GPU BASELINE configs at their full shape.

configs[1]: 256 games, 128x10b bf16, H=8, T=2 x B=16, 800 sims/move: the bench
            workload. Native search (packed rows, 2 pipeline groups of 4096-row
            ResNet launches) vs the callback search (fp32 feature planes through
            NativeNet, 8192 rows per call): identical visit counts and Q for all
            256 games; the schedule's simulation count; no pool overflow; 64
            sampled rows of a real 4096-row launch vs the fp32 restatement.
configs[3]: 256x20b, 1600 sims/move: the same properties at the benched shape
            (256 games, C=256 throughput geometry).
configs[4]: the per-GPU shard of 4096 games over 8 GPUs = 512 games, fp16,
            eval batch 2048 (oamd_engine_set_nn_batch): identical to whole-group
            launches for all 512 games, no overflow.
"""

import numpy as np
import pytest
import torch

import numerics
import resnet_ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
from test_gpu_resnet import LIVE_TOL  # noqa: E402  (per dtype and width: max dpolicy, max dvalue, rms dvalue)


def _bench_sd(C, R, hid):
    """The net bench.py runs for this shape (live init, seed 2025)."""
    import bench

    return bench.bench_state_dict("live", 2025, 17, C, R, hid)


@pytest.fixture(scope="module")
def om():
    import othello_mcts

    return othello_mcts


def _engine(om, G, H, sims, seed):
    b = om.BatchedMCTS(G, history_size=H, num_simulations=sims, num_threads=2, batch_size=16,
                       dirichlet_epsilon=0.25, seed=seed)
    b.random_openings(8, seed=seed + 1)
    return b


def _check_search(om, sd, dtype, G, H, sims, seed, name):
    net = om.NativeNet(sd, device=0, dtype=dtype)
    a = _engine(om, G, H, sims, seed)
    c = _engine(om, G, H, sims, seed)
    sims_a, evals_a = a.search(net)
    sims_c, evals_c = c.search(lambda f: net(f))  # not a NativeNet: the callback path
    L = 32
    assert sims_a == sims_c == G * L * ((sims + L - 1) // L)
    assert evals_a == evals_c and 0 < evals_a <= sims_a
    va, qa = a.root_stats()
    vc, qc = c.root_stats()
    assert torch.equal(va, vc) and torch.equal(qa, qc)
    # every game: root N = the schedule's simulations; children = all but the
    # first round's L selections of the unexpanded root
    info = [a.root_info(g) for g in range(G)]
    assert all(i["visit_count"] == sims_a // G for i in info)
    assert all(sum(i["visit_counts"]) == sims_a // G - L for i in info)
    assert a.engine.status() == (0, 0) and c.engine.status() == (0, 0)
    numerics.record(f"{name} search", f"G={G} sims/game={sims_a // G} native==callback for all games, "
                                      f"nodes/game max={max(i['node_count'] for i in info)}")
    return net, a


def _sampled_launch_rows(om, net, sd, b, G, C_in, dtype, name):
    """A real 4096-row launch (the rows one pipeline group evaluates in a step,
    after a move with tree reuse): 64 sampled non-terminal rows vs the fp32
    restatement (oracle/resnet_ref.py)."""
    b.selfplay_move(temperature_moves=12, opening_moves=0)
    b.engine.search_begin()
    b.engine.select()
    feat = torch.empty((G * 32, C_in, 8, 8), dtype=torch.float32, device=DEV)
    b.engine.features(feat.data_ptr(), 0, G * 32)
    x = feat[:4096].contiguous()
    flags = torch.from_numpy(b.engine.leaf_flags()[:4096].astype(bool))
    out = net(x)
    torch.cuda.synchronize()
    rows = torch.nonzero(flags).flatten()
    pick = rows[torch.randperm(len(rows), generator=torch.Generator().manual_seed(0))[:64]]
    xs = x[pick.to(DEV)].cpu()
    sd_t = {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}
    ref = resnet_ref.forward(sd_t, xs)
    dp = (out["policy"][pick.to(DEV)].cpu() - ref["policy"]).abs().max().item()
    dvs = out["value"][pick.to(DEV)].cpu() - ref["value"]
    dv = dvs.abs().max().item()
    rms = dvs.pow(2).mean().sqrt().item()
    spread = ref["value"].std().item()
    numerics.record(f"{name} 4096-row launch, 64 sampled rows",
                    f"max|dpolicy|={dp:.2e} max|dvalue|={dv:.2e} rms={rms:.2e} (value std over the rows {spread:.3f})")
    assert len(pick) == 64
    assert spread >= 0.05  # the benched net's value is live (it was constant)
    tp, tv, trms = LIVE_TOL[(dtype, sd["conv_block.conv.weight"].shape[0])]
    assert dp <= tp and dv <= tv and rms <= trms
    b.engine.backup()


def test_configs1_full_shape(om):
    sd = _bench_sd(128, 9, 128)
    net, a = _check_search(om, sd, "bf16", 256, 8, 800, 11, "configs[1]")
    b = _engine(om, 256, 8, 800, 12)
    b.search(net)
    _sampled_launch_rows(om, net, sd, b, 256, 17, "bf16", "configs[1]")


def test_configs3_benched_shape(om):
    """configs[3] at the shape the bench runs it (256 games of 256x20b, 1600
    sims/move): 4096-row launches in the C=256 throughput geometry, whose
    register-queue weight stream crosses all 39 conv layers. Native ==
    callback for every game, no pool overflow, and 64 rows of a real launch vs
    the fp32 restatement."""
    sd = _bench_sd(256, 19, 256)
    net, a = _check_search(om, sd, "bf16", 256, 8, 1600, 21, "configs[3]")
    _sampled_launch_rows(om, net, sd, a, 256, 17, "bf16", "configs[3]")


def test_configs4_shard(om):
    net = om.NativeNet(_bench_sd(128, 9, 128), device=0, dtype="fp16")
    runs = []
    for rows in (2048, 0):
        b = _engine(om, 512, 8, 800, 31)
        b.engine.set_nn_batch(rows)
        sims, evals = b.search(net)
        assert sims == 512 * 800
        assert b.engine.status() == (0, 0)
        v, q = b.root_stats()
        runs.append((v.cpu(), q.cpu()))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])
    numerics.record("configs[4] shard", "512 games fp16: eval batch 2048 == whole-group launches")


def test_configs1_tree_vs_oracle_full_shape(om):
    """configs[1]'s tree at full shape against the oracle:
    256 games, H=8, T=2 x B=16, 800 sims, eps=0.25 (Dirichlet noise from each
    game's random stream), 8192-row k_tree rounds through the step API with
    the equivariant stub, 2 moves with tree reuse after 0-8
    random opening plies. A fixed subset of 64 games is replayed by
    OracleMCTS(game_key=...) (oracle/omcts_oracle.c, pinned by the compiled
    reference's fixtures): visit counts, Q bits and the 8-fold self_play_data
    per move. The native search at this shape equals this callback search
    (test_configs1_full_shape), which closes the chain for the bench path.
    Reference: search_thread.cpp:59-260, mcts.cpp:45-165."""
    import oracle as O

    G, H, L = 256, 8, 32
    b = om.BatchedMCTS(G, history_size=H, num_simulations=800, num_threads=2, batch_size=16,
                       dirichlet_epsilon=0.25, seed=303)
    rng = np.random.default_rng(404)
    subset = sorted(rng.choice(G, 64, replace=False).tolist())
    refs = {g: O.OracleMCTS(history_size=H, num_simulations=800, num_threads=2, batch_size=16,
                            dirichlet_epsilon=0.25, game_key=b.engine.game_key(g)) for g in subset}
    # random openings from the host, applied to the engine and to the oracles
    plies = rng.integers(0, 9, G)
    for k in range(int(plies.max())):
        acts = torch.full((G,), -1, dtype=torch.int32)
        for g in range(G):
            if k < plies[g]:
                legal = O.legal_actions(_pos(b, g))
                acts[g] = int(legal[rng.integers(len(legal))])
                if g in refs:
                    refs[g].apply_action(int(acts[g]))
        b.apply_actions(acts.to(DEV))

    def stub(features):
        p, v = O.equivariant_stub(features.cpu().numpy())
        return {"policy": torch.from_numpy(p), "value": torch.from_numpy(v)}

    for mv in range(2):
        sims, evals = b.search(stub)
        assert sims == G * 800 and 0 < evals <= sims
        acts = torch.full((G,), -1, dtype=torch.int32)
        for g, r in refs.items():
            r.search(O.equivariant_stub)
            info = b.root_info(g)
            assert info["visit_counts"] == r.visit_counts(), (mv, g)
            np.testing.assert_array_equal(np.array(info["mean_action_values"], np.float32),
                                          np.array(r.mean_action_values(), np.float32))
            d = b.self_play_data(g)
            f, p = r.self_play_data()
            np.testing.assert_array_equal(torch.stack(d["features"]).numpy(), f)
            np.testing.assert_array_equal(torch.stack(d["policy"]).numpy(), p)
            vc = r.visit_counts()
            acts[g] = O.legal_actions(r.position())[int(np.argmax(vc))]
            r.apply_action(int(acts[g]))
        v, _ = b.root_stats()
        for g in range(G):  # the other games move too (argmax of their visits)
            if g not in refs:
                row = v[g].cpu().numpy()
                acts[g] = int(np.argmax(row)) if row.max() > 0 else -1
        b.apply_actions(acts.to(DEV))
    assert b.engine.status() == (0, 0)
    numerics.record("configs[1] tree vs oracle", f"G={G}, 64 games replayed by the oracle: 2 moves, visits, Q bits, "
                                                 "8-fold targets identical")


def _pos(b, g):
    import oracle as O

    i = b.root_info(g)
    return O.CPos(i["player"], i["player1_discs"], i["player2_discs"], i["legal_moves"], i["next_legal_moves"])


@pytest.mark.parametrize("exact", [True, False], ids=["exact", "round_robin"])
def test_evaluation_lists_through_endgames(om, exact):
    """The native search evaluates only the rows of non-terminal leaves (the
    per-group evaluation lists of tree.hip append_rows, read by the ResNet
    launch): through whole games, restarts and endgames full of terminal
    leaves it must give every game the same visits and Q as the callback path,
    which evaluates every row. 64 games = 2 pipeline groups of 1024-row
    throughput launches; eval batch 384 splits them at list offsets."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(41, 9, 128, 1, 32), device=0)
    kw = dict(history_size=4, num_simulations=64, num_threads=2, batch_size=16, dirichlet_epsilon=0.25, seed=5,
              node_capacity=1 << 16)
    a, c, e = om.BatchedMCTS(64, **kw), om.BatchedMCTS(64, **kw), om.BatchedMCTS(64, **kw)
    e.engine.set_nn_batch(384)
    if not exact:  # all-terminal batches wait for their round (oamd_engine_set_exact_interleaving)
        for x in (a, c, e):
            x.engine.set_exact_interleaving(False)
    for x in (a, c, e):
        x.random_openings(8, seed=6)
    total_sims = total_evals = 0
    for mv in range(75):
        sa, ea = a.search(net)
        sc, ec = c.search(lambda f: net(f))
        se, ee = e.search(net)
        assert (sa, ea) == (sc, ec) == (se, ee), mv
        total_sims += sa
        total_evals += ea
        va, qa = a.root_stats()
        vc, qc = c.root_stats()
        ve, qe = e.root_stats()
        assert torch.equal(va, vc) and torch.equal(qa, qc), mv
        assert torch.equal(va, ve) and torch.equal(qa, qe), mv
        xa = a.selfplay_move(temperature_moves=12, opening_moves=4)["actions"]
        xc = c.selfplay_move(temperature_moves=12, opening_moves=4)["actions"]
        xe = e.selfplay_move(temperature_moves=12, opening_moves=4)["actions"]
        assert torch.equal(xa, xc) and torch.equal(xa, xe), mv
    share = 1.0 - total_evals / total_sims
    numerics.record(f"evaluation lists ({'exact' if exact else 'round-robin'} endgames)",
                    f"64 games x 75 moves: terminal-leaf share {share:.3f}, "
                    "native (lists, eval batch 0 / 384) == callback")
    assert share > 0.02  # the endgames were reached


@pytest.mark.parametrize("G,pipeline", [(256, 0), (96, 3), (8, 0)])
def test_selfplay_steps_equal_move_by_move(om, G, pipeline):
    """oamd_engine_selfplay_steps (each pipeline group chains its searches and
    moves on its own stream) == n x (search + selfplay_move): actions, finish
    codes, 8-fold targets and the trees after the last move, bit for bit;
    G=8 runs one group (the plain call sequence)."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(31, 9, 128, 2, 64), device=0)
    n = 6

    def engine():
        b = om.BatchedMCTS(G, history_size=4, num_simulations=96, num_threads=2, batch_size=16, seed=G,
                           node_capacity=1 << 15)
        b.random_openings(55, seed=5)  # late openings: games end and restart inside the n moves
        if pipeline:
            b.engine.set_pipeline(pipeline)
        return b

    a = engine()
    acts, fins, feats, pols = [], [], [], []
    for _ in range(n):
        a.search(net, sync=False)
        o = a.selfplay_move(temperature_moves=12, opening_moves=4, emit_targets=True)
        acts.append(o["actions"].clone())
        fins.append(o["finished"].clone())
        feats.append(o["features"].clone())
        pols.append(o["policy"].clone())
    b = engine()
    o = b.selfplay_steps(net, n, temperature_moves=12, opening_moves=4, emit_targets=True)
    torch.cuda.synchronize()
    assert torch.equal(o["actions"], torch.stack(acts)) and torch.equal(o["finished"], torch.stack(fins))
    assert torch.equal(o["features"], torch.stack(feats)) and torch.equal(o["policy"], torch.stack(pols))
    va, qa = a.root_stats()
    vb, qb = b.root_stats()
    assert torch.equal(va, vb) and torch.equal(qa, qb)
    restarts = int(((torch.stack(fins) & 3) != 0).sum())
    assert a.engine.status() == (0, 0) and b.engine.status() == (0, 0)
    if G >= 96:
        assert restarts > 0
    numerics.record(f"selfplay_steps G={G} pipeline={pipeline or 'auto'}",
                    f"{n} moves identical to search + selfplay_move, {restarts} game ends")


def test_wide_and_capped_tree_kernels_agree(om):
    """k_tree_wide (launches of <= 16 games, no register cap) and k_tree (the
    96-VGPR cap) run the same rounds: 32 games as one pipeline group (k_tree)
    and as 2 or 4 groups (k_tree_wide), with root noise (the drawn-ahead noise
    windows) and endings inside the moves: actions, finish codes and trees
    equal bit for bit."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(37, 9, 128, 2, 64), device=0)
    outs = {}
    for pipeline in (1, 2, 4):
        b = om.BatchedMCTS(32, history_size=4, num_simulations=160, num_threads=2, batch_size=8, seed=19,
                           dirichlet_epsilon=0.25, node_capacity=1 << 15)
        b.random_openings(53, seed=23)  # 7 empties: games end within the 8 moves
        b.engine.set_pipeline(pipeline)
        acts, fins = [], []
        for _ in range(8):
            b.search(net, sync=False)
            o = b.selfplay_move(temperature_moves=12, opening_moves=4)
            acts.append(o["actions"].clone())
            fins.append(o["finished"].clone())
        torch.cuda.synchronize()
        assert b.engine.status() == (0, 0)
        outs[pipeline] = (torch.stack(acts), torch.stack(fins), *b.root_stats())
    for pipeline in (2, 4):
        for x, y in zip(outs[1], outs[pipeline]):
            assert torch.equal(x, y), pipeline
    ends = int(((outs[1][1] & 3) != 0).sum())
    assert ends > 0
    numerics.record("k_tree_wide == k_tree", f"32 games x 8 moves, eps 0.25, {ends} game ends, groups of 32 / 16 / 8")


@pytest.mark.parametrize("T,B,nn_batch,pipeline,exact", [(3, 8, 0, 0, True), (4, 4, 384, 3, True),
                                                         (2, 16, 0, 0, False)])
def test_free_running_schedules_equal_lock_step(om, T, B, nn_batch, pipeline, exact):
    """Free-running games against the lock-step call for other schedules: 3 and
    4 virtual threads, an NN evaluation batch of 384 rows over 3 pipeline
    groups, round-robin endgames. Actions, finish codes, targets and trees."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(35, 9, 128, 2, 64), device=0)

    def engine(free):
        b = om.BatchedMCTS(96, history_size=4, num_simulations=120, num_threads=T, batch_size=B, seed=11,
                           node_capacity=1 << 16)
        b.random_openings(53, seed=13)  # 7 empties: games end within the 10 moves
        b.engine.set_free_running(free)
        b.engine.set_nn_batch(nn_batch)
        b.engine.set_pipeline(pipeline)
        b.engine.set_exact_interleaving(exact)
        return b

    a, c = engine(True), engine(False)
    oa = a.selfplay_steps(net, 10, temperature_moves=12, opening_moves=4, emit_targets=True)
    oc = c.selfplay_steps(net, 10, temperature_moves=12, opening_moves=4, emit_targets=True)
    torch.cuda.synchronize()
    for k in ("actions", "finished", "features", "policy"):
        assert torch.equal(oa[k], oc[k]), k
    va, qa = a.root_stats()
    vc, qc = c.root_stats()
    assert torch.equal(va, vc) and torch.equal(qa, qc)
    assert int(((oa["finished"] & 3) != 0).sum()) > 0
    assert a.engine.status() == (0, 0)


@pytest.mark.parametrize("keep_all", [True, False])
def test_free_running_games_equal_lock_step(om, keep_all):
    """Free-running self-play (tree.hip k_tree_free, the default of
    selfplay_steps): a game's move runs in the round its search completes and
    its next search starts there, so games near their end (all-terminal
    chains, cut every 2 re-selections) lag the others by rounds. Per game the
    operations are those of n x (search + selfplay_move): actions, finish
    codes, 8-fold targets and the final trees equal the lock-step call's and
    the move-by-move calls' bit for bit; games end and restart inside the call."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(33, 9, 128, 2, 64), device=0)
    n, G = 14, 128

    def engine(free=True):
        b = om.BatchedMCTS(G, history_size=4, num_simulations=160, num_threads=2, batch_size=8, seed=7,
                           node_capacity=1 << 16)
        b.random_openings(50, seed=3)  # late games: chains, endings and restarts inside the call
        b.engine.set_free_running(free)
        return b

    a, c, m = engine(True), engine(False), engine(True)
    oa = a.selfplay_steps(net, n, temperature_moves=12, opening_moves=4, emit_targets=True, keep_all=keep_all)
    oc = c.selfplay_steps(net, n, temperature_moves=12, opening_moves=4, emit_targets=True, keep_all=keep_all)
    outs = []
    for _ in range(n):
        m.search(net, sync=False)
        o = m.selfplay_move(temperature_moves=12, opening_moves=4, emit_targets=True)
        outs.append({k: v.clone() for k, v in o.items()})
    torch.cuda.synchronize()
    om_ = {k: torch.stack([o[k] for o in outs]) if keep_all else outs[-1][k] for k in outs[0]}
    for k in ("actions", "finished", "features", "policy"):
        assert torch.equal(oa[k], oc[k]), k
        assert torch.equal(oa[k], om_[k]), k
    for x, y in ((a, c), (a, m)):
        vx, qx = x.root_stats()
        vy, qy = y.root_stats()
        assert torch.equal(vx, vy) and torch.equal(qx, qy)
    fins = oa["finished"] if keep_all else torch.stack([o["finished"] for o in outs])
    restarts = int(((fins & 3) != 0).sum())
    assert restarts > 0
    sa, ra, _ = a.engine.round_counts()
    sc, rc_, _ = c.engine.round_counts()
    numerics.record(f"free-running games keep_all={keep_all}",
                    f"{G} games x {n} moves identical to lock step and move-by-move; {restarts} game ends; "
                    f"rounds per move free {ra / max(1, sa):.2f} vs lock step {rc_ / max(1, sc):.2f}")
    assert a.engine.status() == (0, 0)


def test_free_running_at_the_benched_shape(om):
    """configs[1] as bench.py runs it (256 games, 128x10b live net, 800 sims,
    random openings, 24 moves in one multi-move call, games ending and
    restarting inside it): free-running games give the lock-step call's
    actions, finish codes and trees bit for bit."""
    import bench

    net = om.NativeNet(bench.bench_state_dict("live", 2025, 17, 128, 9, 128), device=0)
    outs, trees = [], []
    for free in (True, False):
        b = om.BatchedMCTS(256, history_size=8, num_simulations=800, num_threads=2, batch_size=16, seed=2025)
        b.random_openings(40, seed=7)  # late openings: endgames, chains and restarts inside the call
        b.engine.set_free_running(free)
        o = b.selfplay_steps(net, 24, temperature_moves=12, opening_moves=8, emit_targets=False)
        torch.cuda.synchronize()
        outs.append(o)
        trees.append(b.root_stats())
        assert b.engine.status() == (0, 0)
    assert torch.equal(outs[0]["actions"], outs[1]["actions"]) and torch.equal(outs[0]["finished"], outs[1]["finished"])
    assert torch.equal(trees[0][0], trees[1][0]) and torch.equal(trees[0][1], trees[1][1])
    ends = int(((outs[0]["finished"] & 3) != 0).sum())
    assert ends > 10
    numerics.record("free-running games, configs[1] shape", f"256 games x 24 moves == lock step; {ends} game ends")


def test_chain_split_keeps_every_game_identical(om):
    """Chain splitting (oamd_engine_set_chain_split): near a game's end a thread
    whose batches come back all terminal re-selects at once (the reference's
    order) and the native search may stop such a chain and resume it in the
    game's next round. Games late in their play, 10 batches per thread and
    search: budgets 1 and 4 (and no splitting) give the callback path's visits,
    Q, moves and finish codes move after move."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(43, 9, 128, 1, 32), device=0)
    kw = dict(history_size=4, num_simulations=320, num_threads=2, batch_size=16, dirichlet_epsilon=0.25, seed=8,
              node_capacity=1 << 17)
    # (budget, cuts, extra-round grid, adaptive minimum): the extra rounds'
    # ResNet launches loop over the lagging games' rows on a small grid (1
    # workgroup: every board group in turn) or use the regular grid (0); the
    # extra-round count X adapts per search (minimum 0, 1 or 2) or stays at
    # cuts (None)
    splits = [(0, 0, 128, 0), (1, 3, 128, 2), (4, 4, 128, None), (4, 8, 1, 0), (1, 8, 0, None), (1, 16, 128, 1)]
    engines = [om.BatchedMCTS(64, **kw) for _ in splits]
    for x, (budget, cuts, grid, amin) in zip(engines, splits):
        x.engine.set_chain_split(budget, cuts)
        x.engine.set_extra_round_grid(grid)
        x.engine.set_adaptive_extra_rounds(amin is not None, amin or 0)
    ref = om.BatchedMCTS(64, **kw)
    for x in engines + [ref]:
        x.random_openings(50, seed=9)
    total_sims = total_evals = 0
    for mv in range(24):
        sr, er = ref.search(lambda f: net(f))
        total_sims += sr
        total_evals += er
        vr, qr = ref.root_stats()
        xr = ref.selfplay_move(temperature_moves=12, opening_moves=50)
        for x, sp in zip(engines, splits):
            assert x.search(net) == (sr, er), (mv, sp)
            v, q = x.root_stats()
            assert torch.equal(v, vr) and torch.equal(q, qr), (mv, sp)
            o = x.selfplay_move(temperature_moves=12, opening_moves=50)
            assert torch.equal(o["actions"], xr["actions"]) and torch.equal(o["finished"], xr["finished"]), (mv, sp)
    share = 1.0 - total_evals / total_sims
    # the fixed count runs exactly cuts extra rounds (10 batches per thread
    # and search); these late games are in the adaptive count's endgame
    rounds = {sp: x.engine.round_counts() for x, sp in zip(engines, splits)}
    assert rounds[(4, 4, 128, None)][:2] == (24, 24 * 14) and rounds[(1, 8, 0, None)][:2] == (24, 24 * 18)
    n, r, _ = rounds[(1, 16, 128, 1)]
    assert n == 24 and 24 * 11 <= r <= 24 * 26
    numerics.record("chain split", f"64 late games x 24 moves: terminal-leaf share {share:.3f}, "
                                   "budgets 0/1/4, extra-round grids 1/128/regular, fixed and adaptive extra "
                                   f"rounds (budget 1, <= 16 cuts: {r / n - 10:.2f} per search) == callback")
    assert share > 0.1


@pytest.mark.parametrize("opening", [4, 50])
def test_adaptive_extra_rounds(om, opening):
    """The adaptive extra-round count (capi.hip pick_extra_rounds): the first
    two searches run the minimum (0 here: nothing read back yet); from the
    third on, early games (4-ply openings: no terminal leaf, no cut) run none,
    games within 12 empty squares of the end (openings of 0-50 plies over 256
    games: some game is) the full count. Through
    the multi-move self-play call (one pipeline group per stream), the moves
    equal those of the fixed count."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(46, 9, 128, 1, 32), device=0)
    kw = dict(history_size=4, num_simulations=320, num_threads=2, batch_size=16, dirichlet_epsilon=0.25, seed=12,
              node_capacity=1 << 17)
    runs = []
    for adaptive in (True, False):
        x = om.BatchedMCTS(256, **kw)
        x.engine.set_free_running(False)  # the lock-step multi-move call runs the extra rounds
        x.engine.set_chain_split(4, 16)
        x.engine.set_adaptive_extra_rounds(adaptive, 0)
        x.random_openings(opening, seed=13)
        out = x.selfplay_steps(net, 6, temperature_moves=12, opening_moves=opening, emit_targets=True)
        torch.cuda.synchronize()
        runs.append((x.engine.round_counts(), out))
    (n, r, _), out = runs[0]
    (nf, rf, _), out_f = runs[1]
    # 10 batches per thread: 20 per game and search, so at most 20 / 4 = 5
    # cuts, 5 extra rounds (capi.hip extra_rounds), whatever chain_cuts says
    assert n == nf == 6 and rf == 6 * 15
    assert r == (6 * 10 if opening == 4 else 2 * 10 + 4 * 15), (opening, r)
    for k in out:
        assert torch.equal(out[k], out_f[k]), k
    numerics.record(f"adaptive extra rounds, {opening}-ply openings", f"{r - 60} extra rounds in 6 searches "
                    f"(fixed: {rf - 60}); moves and targets identical")


def test_chain_split_with_more_than_64_threads(om):
    """T = 128 virtual threads (one wave serves them in turn): a chain split in
    a search's first round leaves threads unvisited, and every one of them
    must still start the search fresh (k_tree resets the per-thread state with
    a strided loop). Late games, budget 1: the split search equals
    the unsplit callback path move after move."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(44, 9, 128, 1, 32), device=0)
    kw = dict(history_size=4, num_simulations=1536, num_threads=128, batch_size=4, dirichlet_epsilon=0.25,
              seed=18, node_capacity=1 << 18)
    x = om.BatchedMCTS(16, **kw)
    x.engine.set_chain_split(1, 3)
    ref = om.BatchedMCTS(16, **kw)
    for b in (x, ref):
        b.random_openings(50, seed=19)
    total_sims = total_evals = 0
    for mv in range(8):
        sr, er = ref.search(lambda f: net(f))
        total_sims += sr
        total_evals += er
        assert x.search(net) == (sr, er), mv
        vr, qr = ref.root_stats()
        v, q = x.root_stats()
        assert torch.equal(v, vr) and torch.equal(q, qr), mv
        o = x.selfplay_move(temperature_moves=12, opening_moves=50)
        orf = ref.selfplay_move(temperature_moves=12, opening_moves=50)
        assert torch.equal(o["actions"], orf["actions"]) and torch.equal(o["finished"], orf["finished"]), mv
    numerics.record("chain split T=128", f"16 late games x 8 moves: terminal-leaf share "
                                         f"{1.0 - total_evals / total_sims:.3f}, budget 1 == callback")
    assert total_evals < total_sims


def test_more_than_65535_batches_per_thread(om):
    """steps = ceil(S / L) has no upper limit (1 leaf per step, 70,000
    simulations): the per-thread batch count must not run into the
    waiting-for-NN flag. Every simulation reaches the root."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(45, 9, 128, 1, 32), device=0)
    b = om.BatchedMCTS(2, history_size=4, num_simulations=70000, num_threads=1, batch_size=1,
                       dirichlet_epsilon=0.0, seed=3, node_capacity=1 << 21)
    sims, evals = b.search(net)
    assert sims == 2 * 70000
    for g in range(2):
        info = b.root_info(g)
        assert info["visit_count"] == 70000
        assert sum(info["visit_counts"]) == 70000 - 1  # the first leaf is the unexpanded root
    assert b.engine.status() == (0, 0)


def test_tree_work_counters_price_the_byte_model(om):
    """the counters bench.py prices with SURVEY §8(d)'s
    per-item bytes (oamd_engine_tree_work) count what the tree kernels did:
    levels = the summed descent depths, children created = the games' node
    count growth, an expansion creates >= 1 child and needs an evaluated
    leaf, every descent level scans >= 1 child, one count per tree launch."""
    from othello_mcts.synthetic import live_state_dict

    net = om.NativeNet(live_state_dict(5, 17, 128, 2, 32), device=0)
    b = _engine(om, 64, 8, 256, 41)
    nodes0 = sum(b.root_info(g)["node_count"] for g in range(64))
    lv0, sc0, ex0, cr0, la0 = b.engine.tree_work()
    _, ds0, _ = b.engine.descent_depths()
    sims, evals = b.search(net)
    lv1, sc1, ex1, cr1, la1 = b.engine.tree_work()
    _, ds1, _ = b.engine.descent_depths()
    nodes1 = sum(b.root_info(g)["node_count"] for g in range(64))
    assert lv1 - lv0 == ds1 - ds0 > 0
    assert cr1 - cr0 == nodes1 - nodes0 > 0
    assert 0 < ex1 - ex0 <= evals and ex1 - ex0 <= cr1 - cr0
    assert sc1 - sc0 >= lv1 - lv0
    steps = 256 // 32
    assert la1 - la0 >= steps  # >= one launch per round (2 pipeline groups: 2 per round + final backups)
    numerics.record("tree work counters", f"levels={lv1 - lv0} scanned={sc1 - sc0} expansions={ex1 - ex0} "
                                          f"children={cr1 - cr0} launches={la1 - la0} sims={sims} evals={evals}")

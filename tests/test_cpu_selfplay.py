"""Host logic of the self-play data path and checkpoint ingest (no GPU).

SelfPlayCollector restates train.py:438-450 (value targets) over the
selfplay_move output stream; load_checkpoint restates player.py:195-228."""

import json

import pytest
import torch

from othello_mcts.selfplay import FIN_BLACK, FIN_DRAW, FIN_NONE, FIN_WHITE, SelfPlayCollector


def _move(G, C, black_to_move, actions, finished, tag):
    f = torch.zeros((G, 8, C, 8, 8))
    p = torch.zeros((G, 8, 65))
    for g in range(G):
        f[g, :, 0] = 0.0 if black_to_move[g] else 1.0  # plane 0 = player - 1
        f[g, :, 1, 0, 0] = tag  # identifies the move
        p[g, :, 0] = tag
    return {"actions": torch.tensor(actions, dtype=torch.int32), "finished": torch.tensor(finished, dtype=torch.int32),
            "features": f, "policy": p}


def test_collector_values_follow_reference_rule():
    col = SelfPlayCollector(2)
    # game 0: black, white, white (a pass by black in between), then black wins
    assert col.add(_move(2, 5, [True, True], [19, 26], [FIN_NONE, FIN_NONE], 1.0)) == \
        {"features": [], "policies": [], "values": []}
    col.add(_move(2, 5, [False, False], [18, 20], [FIN_NONE, FIN_NONE], 2.0))
    col.add(_move(2, 5, [True, False], [64, 21], [FIN_NONE, FIN_NONE], 3.0))
    out = col.add(_move(2, 5, [False, True], [40, 22], [FIN_BLACK, FIN_NONE], 4.0))
    assert len(out["features"]) == len(out["policies"]) == len(out["values"]) == 4 * 8
    vals = [float(v) for v in out["values"]]
    # reference: +outcome at step 0, alternating every step (passes count as steps)
    ref = []
    v = 1.0
    while len(ref) < 32:
        ref += [v] * 8
        v = -v
    assert vals == ref
    assert [float(f[1, 0, 0]) for f in out["features"][::8]] == [1.0, 2.0, 3.0, 4.0]
    assert [float(p[0]) for p in out["policies"][::8]] == [1.0, 2.0, 3.0, 4.0]
    assert col.games_completed == 1 and col.pending_moves(0) == 0 and col.pending_moves(1) == 4
    # game 1: white won; a slot without a searched root (action -1) adds no sample
    col.add(_move(2, 5, [True, True], [-1, 23], [FIN_NONE, FIN_NONE], 5.0))
    out = col.add(_move(2, 5, [True, False], [-1, 24], [FIN_NONE, FIN_WHITE], 6.0))
    vals = [float(v) for v in out["values"][::8]]
    # game 1 steps: black, white, white, black, black, white to move -> white won
    assert vals == [-1.0, 1.0, 1.0, -1.0, -1.0, 1.0]
    assert col.pending_moves(0) == 0


def test_collector_draw_and_errors():
    col = SelfPlayCollector(1)
    out = col.add(_move(1, 3, [False], [5], [FIN_DRAW], 1.0))
    assert [float(v) for v in out["values"]] == [0.0] * 8
    with pytest.raises(ValueError):
        col.add({"actions": torch.zeros(1, dtype=torch.int32), "finished": torch.zeros(1, dtype=torch.int32)})
    with pytest.raises(ValueError):
        col.add(_move(2, 3, [True, True], [1, 1], [0, 0], 0.0))


def test_load_checkpoint_roundtrip_and_validation(tmp_path):
    from othello_mcts.native import load_checkpoint
    from othello_mcts.synthetic import alphazero_state_dict, net_config_from_state_dict

    sd = {k: torch.from_numpy(v) for k, v in alphazero_state_dict(3, 9, 128, 2, 32).items()}
    cfg = net_config_from_state_dict(sd)
    d = tmp_path / "007"
    d.mkdir()
    torch.save(sd, d / "neural_net.pth")
    (d / "config.json").write_text(json.dumps({"neural_net": cfg, "mcts": {"history_size": 4}}))
    config, sd2 = load_checkpoint(d)
    assert config["neural_net"] == cfg
    assert sd2.keys() == sd.keys() and all(torch.equal(sd[k], sd2[k]) for k in sd)

    bad = dict(cfg, in_channels=8)
    (d / "config.json").write_text(json.dumps({"neural_net": bad}))
    with pytest.raises(ValueError, match="Expected in_channels to be odd, but got 8."):
        load_checkpoint(d)
    (d / "config.json").write_text(json.dumps({"neural_net": dict(cfg, in_channels=1)}))
    with pytest.raises(ValueError, match="Expected history_size to be positive, but got 0."):
        load_checkpoint(d)
    (d / "config.json").write_text(json.dumps({"neural_net": dict(cfg, conv_channels=256)}))
    with pytest.raises(ValueError, match="conv_channels"):
        load_checkpoint(d)


@pytest.mark.parametrize("gi", [0, 1])
def test_collector_reproduces_reference_self_play_samples(gi):
    """Feed the reference _self_play game (compiled reference MCTS, tests/golden/
    ref_self_play.*) to SelfPlayCollector as a selfplay_move stream: the samples
    it returns are the reference's, in order — features, policies and value
    targets (train.py:404-452)."""
    import numpy as np

    import ref_fixtures as RF
    from othello_mcts import Position
    from othello_mcts.selfplay import outcome_for_black

    games, arr = RF.load_self_play()
    g = games[gi]
    f_exp, p_exp, v_exp = RF.self_play_expected(games, arr, gi)
    pos = Position.initial_position()
    for a in g["actions"]:
        pos = pos.apply_action(a)
    assert pos.is_terminal()
    fin = {1.0: FIN_BLACK, -1.0: FIN_WHITE, 0.0: FIN_DRAW}[outcome_for_black(pos.player1_discs(),
                                                                             pos.player2_discs())]
    col = SelfPlayCollector(1)
    n = len(g["actions"])
    for t, a in enumerate(g["actions"]):
        out = col.add({"actions": torch.tensor([a], dtype=torch.int32),
                       "finished": torch.tensor([fin if t == n - 1 else FIN_NONE], dtype=torch.int32),
                       "features": torch.from_numpy(f_exp[8 * t: 8 * t + 8])[None],
                       "policy": torch.from_numpy(p_exp[8 * t: 8 * t + 8])[None]})
    assert len(out["values"]) == 8 * n
    np.testing.assert_array_equal(torch.stack(out["features"]).numpy(), f_exp)
    np.testing.assert_array_equal(torch.stack(out["policies"]).numpy(), p_exp)
    np.testing.assert_array_equal(torch.stack(out["values"]).numpy(), v_exp)

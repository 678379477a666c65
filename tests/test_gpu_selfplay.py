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
    assert (out["value"] - ref["value"]).abs().max().item() <= 3e-2

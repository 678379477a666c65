"""Native ResNet (csrc/resnet.hip) parity on the GPU.

Yardsticks: the reference's own AlphaZeroNet outputs (tests/golden/resnet.npz,
fp32 torch CPU) and the fp32 torch restatement (oracle/resnet_ref.py) on the
same inputs. The kernel computes in bf16 (or fp16) with fp32 accumulation and
fp32 heads. Two sets of tolerances (absolute, on probabilities / tanh values):
  * TOL, for the torch-default-init goldens (rounds 1-2's nets, whose 10-block
    tower forgets its input, so the value barely moves): bf16 policy <= 5e-4,
    value <= 3e-3; fp16 policy <= 1e-4, value <= 1e-3 (about 3-5x the
    largest errors measured on those nets). They do NOT describe a live net.
  * LIVE_TOL, for the nets bench.py runs and the self-play trained net (live
    value heads): per dtype and tower width, max |dpolicy|, max |dvalue| and
    rms dvalue — bf16 value errors reach 0.067 (C=128) and 0.114 (C=256) there
    (see the block above LIVE_TOL). What those errors do to the search is
    measured in tests/test_gpu_search_dtype.py.
Every case's measured maxima are printed in the terminal summary (numerics.py).
"""

import json

import numpy as np
import pytest
import torch

import numerics
import resnet_ref

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
TOL = {"bf16": (5e-4, 3e-3), "fp16": (1e-4, 1e-3)}


@pytest.fixture(scope="module")
def om():
    import othello_mcts

    return othello_mcts


def _sd(meta):
    from othello_mcts.synthetic import alphazero_state_dict

    return alphazero_state_dict(meta["seed"], 1 + 2 * meta["history_size"], meta["conv_channels"],
                                meta["num_residual_blocks"], meta["value_head_hidden_channels"])


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("name", ["c128b9_h8", "c128b9_h4", "c256b19_h8"])
def test_native_net_vs_reference_golden(om, golden_dir, name, dtype):
    meta = json.loads((golden_dir / "resnet_meta.json").read_text())[name]
    g = np.load(golden_dir / "resnet.npz")
    net = om.NativeNet(_sd(meta), device=0, dtype=dtype)
    x = torch.from_numpy(g[f"{name}_x"].astype(np.float32)).to(DEV)
    out = net(x)
    torch.cuda.synchronize()
    dp = np.abs(out["policy"].cpu().numpy() - g[f"{name}_policy"]).max()
    dv = np.abs(out["value"].cpu().numpy() - g[f"{name}_value"]).max()
    numerics.record(f"resnet golden {name} {dtype}", f"max|dpolicy|={dp:.2e} max|dvalue|={dv:.2e}")
    tp, tv = TOL[dtype]
    assert dp <= tp and dv <= tv


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("name", ["c128b9_h8_r1027", "c128b9_h4_r1029", "c256b19_h8_r1025"])
def test_throughput_geometry_vs_reference_golden(om, golden_dir, name, dtype):
    """The geometries every bench launch runs (>= 1024 rows: 4-board C=128
    workgroups with the LDS weight ring, 2-board C=256 workgroups with the
    register-queue weight stream across all 39 convs) against the reference's
    own AlphaZeroNet (neural_net.py:138-172) on >= 1025 real positions, ragged
    in the last workgroup. The planes are regenerated from their seed
    (ref_fixtures.real_features) and checked against the stored checksum."""
    from ref_fixtures import planes_checksum, real_features

    meta = json.loads((golden_dir / "resnet_large_meta.json").read_text())[name]
    g = np.load(golden_dir / "resnet_large.npz")
    x = real_features(meta["boards"], meta["history_size"], meta["planes_seed"])
    assert planes_checksum(x) == meta["planes_sha256_16"]
    assert len(x) >= 1024  # resnet.hip kSmallBatchRows: the throughput geometry
    net = om.NativeNet(_sd(meta), device=0, dtype=dtype)
    out = net(torch.from_numpy(x).to(DEV))
    torch.cuda.synchronize()
    dp = np.abs(out["policy"].cpu().numpy() - g[f"{name}_policy"]).max()
    dv = np.abs(out["value"].cpu().numpy() - g[f"{name}_value"]).max()
    numerics.record(f"resnet golden {name} {dtype} (throughput geometry)",
                    f"max|dpolicy|={dp:.2e} max|dvalue|={dv:.2e}")
    tp, tv = TOL[dtype]
    assert dp <= tp and dv <= tv


# live nets (value spread ~0.5, priors up to peaked): the bf16 (fp16)
# rounding of the tower's activations between its 19 convs dominates (an fp32
# emulation of the kernel's roundings reproduces the GPU's errors: value rms
# 0.0135, max 0.062 at bf16), so these tolerances are their own:
# max |dpolicy|, max |dvalue|, rms dvalue, per dtype and tower depth (19 / 39
# convs; measured C=128 bf16 8e-4-2.5e-3 / 0.057-0.067 / 0.0135-0.014, fp16
# 2.2e-4-3.3e-4 / 0.0074-0.0085 / 0.0017-0.0019; C=256 bf16 2.4e-3 / 0.114 /
# 0.0247; the self-play trained net's priors reach 0.99, its bf16 policy error
# 1.17e-2, value 0.025 / rms 0.0034)
LIVE_TOL = {("bf16", 128): (2.5e-2, 1e-1, 2.5e-2), ("fp16", 128): (4e-3, 2e-2, 5e-3),
            ("bf16", 256): (5e-3, 2e-1, 4e-2), ("fp16", 256): (1e-3, 4e-2, 8e-3)}


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("name", ["live_c128b9_h8_r1027", "frontier_c128b9_h8_r1027", "selfplay_c128b9_h8_r1027",
                                  "live_c256b19_h8_r1025"])
def test_live_nets_vs_reference_golden(om, name, dtype):
    """The nets bench.py runs (live value heads, the deep_tree
    net's peaked priors) against the reference's own AlphaZeroNet on >= 1025
    real positions in the throughput geometries (make_golden.py
    make_resnet_live; weights and planes regenerated, checksum-checked)."""
    import ref_fixtures as RF

    meta, sd, x, g = RF.live_case(name)
    net = om.NativeNet(sd, device=0, dtype=dtype)
    out = net(torch.from_numpy(x).to(DEV))
    torch.cuda.synchronize()
    p, v = out["policy"].cpu().numpy(), out["value"].cpu().numpy()
    dp = np.abs(p - g["policy"]).max()
    dv = np.abs(v - g["value"]).max()
    # relative to the output's own scale: the largest prior / the value spread
    numerics.record(f"resnet live golden {name} {dtype}",
                    f"max|dpolicy|={dp:.2e} max|dvalue|={dv:.2e} (value std {g['value'].std():.3f}, "
                    f"mean max prior {g['policy'].max(1).mean():.3f}, rms dvalue {np.sqrt(((v - g['value'])**2).mean()):.2e})")
    assert v.std() > 0.3  # live on the GPU too
    tp, tv, trms = LIVE_TOL[(dtype, meta["conv_channels"])]
    assert dp <= tp and dv <= tv and np.sqrt(((v - g["value"]) ** 2).mean()) <= trms


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("rows", [1, 3, 4, 5, 257, 1027, 2048])
def test_native_net_vs_torch_fp32_restatement(om, rows, dtype):
    """Ragged batch sizes (partial last workgroup tile) on real-looking planes."""
    from othello_mcts.synthetic import alphazero_state_dict

    sd = alphazero_state_dict(99, 17, 128, 9, 128)
    net = om.NativeNet(sd, device=0, dtype=dtype)
    gen = torch.Generator().manual_seed(rows)
    x = (torch.rand((rows, 17, 8, 8), generator=gen) < 0.3).float()
    x[:, 0] = (torch.rand((rows, 1, 1), generator=gen) < 0.5).float()
    x = x.to(DEV)
    ref = resnet_ref.forward(sd, x)
    out = net(x)
    dp = (out["policy"] - ref["policy"]).abs().max().item()
    dv = (out["value"] - ref["value"]).abs().max().item()
    numerics.record(f"resnet restatement rows={rows} {dtype}", f"max|dpolicy|={dp:.2e} max|dvalue|={dv:.2e}")
    tp, tv = TOL[dtype]
    assert dp <= tp and dv <= tv
    torch.testing.assert_close(out["policy"].sum(1), torch.ones(rows, device=DEV), atol=1e-5, rtol=0)


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_native_net_max_history_vs_restatement(om, dtype):
    """31 input planes (history 15) through the packed-row and fp32 paths."""
    from othello_mcts.synthetic import alphazero_state_dict

    sd = alphazero_state_dict(5, 31, 128, 2, 64)
    net = om.NativeNet(sd, device=0, dtype=dtype)
    gen = torch.Generator().manual_seed(31)
    x = (torch.rand((300, 31, 8, 8), generator=gen) < 0.3).float()
    x[:, 0] = (torch.rand((300, 1, 1), generator=gen) < 0.5).float()
    x = x.to(DEV)
    ref = resnet_ref.forward(sd, x)
    out = net(x)
    tp, tv = TOL[dtype]
    numerics.record(f"resnet history15 {dtype}",
                    f"max|dpolicy|={(out['policy'] - ref['policy']).abs().max().item():.2e} "
                    f"max|dvalue|={(out['value'] - ref['value']).abs().max().item():.2e}")
    assert (out["policy"] - ref["policy"]).abs().max().item() <= tp
    assert (out["value"] - ref["value"]).abs().max().item() <= tv


def test_native_search_equals_callback_search(om):
    """The packed-feature native path and the fp32-feature callback path feed the
    same kernel the same planes: visit counts must agree exactly."""
    from othello_mcts.synthetic import alphazero_state_dict

    sd = alphazero_state_dict(7, 9, 128, 3, 64)
    net = om.NativeNet(sd, device=0)
    kw = dict(history_size=4, num_simulations=128, num_threads=2, batch_size=16, dirichlet_epsilon=0.25,
              seed=21, node_capacity=1 << 16)
    a = om.BatchedMCTS(8, **kw)
    b = om.BatchedMCTS(8, **kw)
    a.random_openings(6, seed=5)
    b.random_openings(6, seed=5)

    def cb(features):
        return net(features)

    for _ in range(3):
        a.search(net)
        b.search(cb)
        for g in range(8):
            assert a.visit_counts(g) == b.visit_counts(g)
            assert a.mean_action_values(g) == b.mean_action_values(g)
        # both engines consume the same random events (move choice, restarts)
        xa = a.selfplay_move(temperature_moves=12, opening_moves=3)["actions"].cpu()
        xb = b.selfplay_move(temperature_moves=12, opening_moves=3)["actions"].cpu()
        assert torch.equal(xa, xb)


@pytest.mark.parametrize("threads,batch", [(2, 16), (3, 8), (4, 4)])
def test_single_game_thread_split_equals_callback_search(om, threads, batch):
    """One game with T > 1 runs the thread-split schedule (thread t's ResNet rows
    on their own stream while the tree kernel serves thread t+1); the callback
    path backs up and selects in the same order through the step API. Visits,
    Q and the move choices must agree exactly, with Dirichlet noise and tree
    reuse."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(11, 9, 128, 2, 32), device=0)
    kw = dict(history_size=4, num_simulations=200, num_threads=threads, batch_size=batch,
              dirichlet_epsilon=0.25, seed=33, node_capacity=1 << 16)
    a = om.BatchedMCTS(1, **kw)
    b = om.BatchedMCTS(1, **kw)
    a.random_openings(6, seed=2)
    b.random_openings(6, seed=2)
    for _ in range(4):
        a.search(net)
        b.search(lambda f: net(f))
        assert a.visit_counts(0) == b.visit_counts(0)
        assert a.mean_action_values(0) == b.mean_action_values(0)
        xa = a.selfplay_move(temperature_moves=12)["actions"].cpu()
        xb = b.selfplay_move(temperature_moves=12)["actions"].cpu()
        assert torch.equal(xa, xb)


def test_mcts_autodetects_alphazero_module(om):
    """MCTS.search(AlphaZeroNet-shaped module) runs the native path, refreshes
    after in-place weight updates, and agrees with NativeNet."""
    from othello_mcts import native
    from othello_mcts.synthetic import alphazero_state_dict

    sd = alphazero_state_dict(8, 9, 128, 1, 32)

    class AlphaZeroNet(torch.nn.Module):  # stands in for neural_net.py:138-172 (stock forward)
        def __init__(self):
            super().__init__()
            self.conv_block = torch.nn.Module()
            self.residual_blocks = torch.nn.Module()
            self.policy_head = torch.nn.Module()
            self.value_head = torch.nn.Module()
            self.params = torch.nn.ParameterDict()
            self._sd = {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}

        def state_dict(self, *a, **k):
            return dict(self._sd)

        def forward(self, x):
            raise AssertionError("replaced by the native kernel")

    class LogitsNet(AlphaZeroNet):  # overrides forward: never replaced
        def forward(self, x):
            return {}

    m = AlphaZeroNet().eval()
    # the drop-in default is fp16 (round 6: closer to the fp32 search than
    # bf16, tests/test_gpu_search_dtype.py), for a net with fp16 headroom
    with pytest.warns(RuntimeWarning, match="fp16"):
        nn1 = native.resolve(m, 0, 4)
    assert nn1 is not None and nn1.dtype == "fp16" and native.resolve(m, 0, 4) is nn1
    assert native.resolve(LogitsNet().eval(), 0, 4) is None
    nnb = native.resolve(m, 0, 4, "bf16")
    assert nnb is not None and nnb.dtype == "bf16"
    # a net whose activations would overflow fp16 is evaluated in bf16
    big = AlphaZeroNet().eval()
    big._sd = {k: (v * 1e4 if k.endswith("conv2.weight") else v) for k, v in big._sd.items()}
    with pytest.warns(RuntimeWarning, match="headroom"):
        nnbig = native.resolve(big, 0, 4)
    assert nnbig.dtype == "bf16"


def test_pipeline_groups_do_not_change_results(om):
    """Splitting the games over 1, 2, 3 or 8 stream groups, and letting the
    groups' ResNet launches run as 1, 2 or 4 concurrent chains
    (oamd_engine_set_nn_chains, bench --nn-chains), are pure scheduling
    choices: every game's visits and Q must be identical."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(17, 9, 128, 2, 32), device=0)
    kw = dict(history_size=4, num_simulations=96, num_threads=2, batch_size=8, seed=9,
              node_capacity=1 << 15)
    runs = []
    for groups, chains in ((1, 1), (2, 1), (3, 1), (8, 1), (2, 2), (4, 2), (8, 4)):
        b = om.BatchedMCTS(12, **kw)
        b.engine.set_pipeline(groups)
        b.engine.set_nn_chains(chains)
        b.random_openings(5, seed=3)
        for _ in range(2):
            b.search(net)
            b.selfplay_move(temperature_moves=12, opening_moves=2)
        b.search(net)
        runs.append([(b.visit_counts(g), b.mean_action_values(g)) for g in range(12)])
    assert all(r == runs[0] for r in runs[1:])


def test_nn_batch_does_not_change_results(om):
    """Evaluating a group's rows in several ResNet launches (oamd_engine_set_nn_batch,
    configs[4]'s eval batch) changes no game's statistics."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(17, 9, 128, 2, 32), device=0)
    kw = dict(history_size=4, num_simulations=96, num_threads=2, batch_size=8, seed=9,
              node_capacity=1 << 15)
    runs = []
    for rows in (0, 64, 100):
        b = om.BatchedMCTS(12, **kw)
        b.engine.set_nn_batch(rows)
        b.random_openings(5, seed=3)
        for _ in range(2):
            b.search(net)
            b.selfplay_move(temperature_moves=12, opening_moves=2)
        b.search(net)
        runs.append([(b.visit_counts(g), b.mean_action_values(g)) for g in range(12)])
    assert runs[0] == runs[1] == runs[2]


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("C,R", [(128, 9), (256, 3), (256, 19)])
def test_small_batch_geometry_is_bit_identical(om, dtype, C, R):
    """Fewer than 1024 rows run one board per workgroup (latency geometry);
    the K order per output is unchanged, so rows evaluated alone match the
    same rows inside a large (throughput-geometry) batch bit for bit. 1101
    rows: the large batch's last workgroup is ragged (1101 = 4 x 275 + 1).
    (256, 19) is configs[3]'s tower: the C=256 register queue runs on across
    all 39 conv layers' boundaries into the zero pad."""
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(11, 17, C, R, 64), device=0, dtype=dtype)
    gen = torch.Generator().manual_seed(C)
    x = (torch.rand((1101, 17, 8, 8), generator=gen) < 0.3).float().to(DEV)
    big = net(x)
    small = net(x[:100].contiguous())
    assert torch.equal(big["policy"][:100], small["policy"])
    assert torch.equal(big["value"][:100], small["value"])
    tail = net(x[1001:].contiguous())  # the ragged last workgroup's board, alone
    assert torch.equal(big["policy"][1001:], tail["policy"])
    assert torch.equal(big["value"][1001:], tail["value"])

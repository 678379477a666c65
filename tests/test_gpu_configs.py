"""The single-GPU BASELINE configs at their full shape.

configs[1]: 256 games, 128x10b bf16, H=8, T=2 x B=16, 800 sims/move: the bench
            workload. Native search (packed rows, 2 pipeline groups of 4096-row
            ResNet launches) vs the callback search (fp32 feature planes through
            NativeNet, 8192 rows per call): identical visit counts and Q for all
            256 games; the schedule's simulation count; no pool overflow; 64
            sampled rows of a real 4096-row launch vs the fp32 restatement.
configs[3]: 256x20b, 1600 sims/move: the same properties on 8 games.
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
TOL = {"bf16": (2e-3, 1e-2), "fp16": (5e-4, 2e-3)}  # as tests/test_gpu_resnet.py


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


def test_configs1_full_shape(om):
    from othello_mcts.synthetic import alphazero_state_dict

    sd = alphazero_state_dict(2025, 17, 128, 9, 128)
    net, a = _check_search(om, sd, "bf16", 256, 8, 800, 11, "configs[1]")
    # a real 4096-row launch: the rows one pipeline group evaluates in a step
    b = _engine(om, 256, 8, 800, 12)
    b.search(net)
    b.selfplay_move(temperature_moves=12, opening_moves=0)
    b.engine.search_begin()
    b.engine.select()
    feat = torch.empty((256 * 32, 17, 8, 8), dtype=torch.float32, device=DEV)
    b.engine.features(feat.data_ptr(), 0, 256 * 32)
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
    dv = (out["value"][pick.to(DEV)].cpu() - ref["value"]).abs().max().item()
    numerics.record("configs[1] 4096-row launch, 64 sampled rows", f"max|dpolicy|={dp:.2e} max|dvalue|={dv:.2e}")
    assert len(pick) == 64
    assert dp <= TOL["bf16"][0] and dv <= TOL["bf16"][1]
    b.engine.backup()


def test_configs3_shape(om):
    from othello_mcts.synthetic import alphazero_state_dict

    sd = alphazero_state_dict(2026, 17, 256, 19, 256)
    _check_search(om, sd, "bf16", 8, 8, 1600, 21, "configs[3]")


def test_configs4_shard(om):
    from othello_mcts.synthetic import alphazero_state_dict

    net = om.NativeNet(alphazero_state_dict(2027, 17, 128, 9, 128), device=0, dtype="fp16")
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

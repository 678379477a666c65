"""Generate the committed golden fixtures (run in the build container only).

Every expected value here is produced by the REFERENCE itself:
  * bitboard / transform / feature / string / error vectors: oracle/_ref/ref_driver,
    compiled from the reference headers where they lie (/root/reference/cpp/src/include,
    see oracle/Makefile target ``ref``);
  * ResNet policy/value vectors: the reference's own ``AlphaZeroNet``
    (/root/reference/python/othello_alphazero/neural_net.py) imported read-only,
    in eval mode, fp32 on CPU, with seeded synthetic weights
    (othello_mcts.synthetic.alphazero_state_dict, regenerable anywhere).
  * MCTS known answers: the visit counts SURVEY.md §4 recorded from the compiled
    reference extension (num_threads=1, dirichlet_epsilon=0, stub nets of
    SURVEY.md Appendix B.3).

Usage:  python tests/golden/make_golden.py
Outputs (small, committed): tests/golden/*.npz, tests/golden/*.json
Nothing from the reference (source, bytecode) is copied into the repository.
"""

from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
GOLD = ROOT / "tests" / "golden"
DRIVER = ROOT / "oracle" / "_ref" / "ref_driver"
REF_PY = Path("/root/reference/python")

sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))


def run(*args: str) -> list[str]:
    out = subprocess.run([str(DRIVER), *args], check=True, capture_output=True, text=True)
    return out.stdout.splitlines()


def u64(h: str) -> int:
    return int(h, 16)


def as_i64(vals) -> np.ndarray:
    return np.array(vals, dtype=np.uint64).view(np.int64)


def make_bitboards() -> None:
    # --- full random games: every position, every child
    pos, lm, children = [], [], []
    for line in run("games", "30", "20250222"):
        f = line.split()
        if f[0] == "P":
            pos.append([int(f[1]), u64(f[2]), u64(f[3]), u64(f[4])])
        elif f[0] == "L":
            lm.append([len(pos) - 1, u64(f[1])])
        elif f[0] == "A":
            children.append(
                [len(pos) - 1, int(f[1]), u64(f[2]), int(f[3]), u64(f[4]), u64(f[5]), u64(f[6])]
            )
    pos_a = np.array(pos, dtype=object)
    ch = np.array(children, dtype=object)
    lm_a = np.array(lm, dtype=object)
    # --- random disjoint boards (unreachable positions stress the edge masks)
    rnd, flips = [], []
    for line in run("random", "4000", "777"):
        f = line.split()
        if f[0] == "R":
            rnd.append([u64(f[1]), u64(f[2]), u64(f[3])])
        else:
            flips.append([len(rnd) - 1, int(f[1]), u64(f[2])])
    rnd_a = np.array(rnd, dtype=object)
    fl = np.array(flips, dtype=object)
    table = []
    for line in run("table"):
        f = line.split()
        table.append([int(x) for x in f[2:]])
    np.savez_compressed(
        GOLD / "bitboards.npz",
        pos_player=pos_a[:, 0].astype(np.int32),
        pos_p1=as_i64(pos_a[:, 1]),
        pos_p2=as_i64(pos_a[:, 2]),
        pos_legal=as_i64(pos_a[:, 3]),
        lm_index=lm_a[:, 0].astype(np.int32),
        lm_value=as_i64(lm_a[:, 1]),
        ch_parent=ch[:, 0].astype(np.int32),
        ch_action=ch[:, 1].astype(np.int32),
        ch_flips=as_i64(ch[:, 2]),
        ch_player=ch[:, 3].astype(np.int32),
        ch_p1=as_i64(ch[:, 4]),
        ch_p2=as_i64(ch[:, 5]),
        ch_legal=as_i64(ch[:, 6]),
        rnd_me=as_i64(rnd_a[:, 0]),
        rnd_opp=as_i64(rnd_a[:, 1]),
        rnd_legal=as_i64(rnd_a[:, 2]),
        fl_index=fl[:, 0].astype(np.int32),
        fl_square=fl[:, 1].astype(np.int32),
        fl_flips=as_i64(fl[:, 2]),
        transform_table=np.array(table, dtype=np.int32),
    )
    print("bitboards:", len(pos), "positions,", len(children), "children,", len(rnd), "random boards")


def make_features() -> None:
    chains, hs, ts, feats = [], [], [], []
    cur = None
    for line in run("features", "120", "4242"):
        f = line.split()
        if f[0] == "C":
            cur = []
            chains.append(cur)
        elif f[0] == "P":
            cur.append([int(f[1]), u64(f[2]), u64(f[3]), u64(f[4])])
        elif f[0] == "X":
            hs.append(int(f[1]))
            ts.append(int(f[2]))
            feats.append(np.array([int(x) for x in f[3:]], dtype=np.int8))
    # flatten: chain_offsets index into a concatenated position table (oldest first)
    offs = np.cumsum([0] + [len(c) for c in chains]).astype(np.int32)
    allp = np.array([p for c in chains for p in c], dtype=object)
    foffs = np.cumsum([0] + [len(x) for x in feats]).astype(np.int32)
    np.savez_compressed(
        GOLD / "features.npz",
        chain_offsets=offs,
        player=allp[:, 0].astype(np.int32),
        p1=as_i64(allp[:, 1]),
        p2=as_i64(allp[:, 2]),
        legal=as_i64(allp[:, 3]),
        history_size=np.array(hs, np.int32),
        transform=np.array(ts, np.int32),
        feat_offsets=foffs,
        features=np.concatenate(feats),
    )
    print("features:", len(chains), "chains")


def make_strings_errors() -> None:
    out = {"strings": [], "errors": {}}
    pend = None
    for line in run("strings", "24", "99"):
        f = line.split()
        if f[0] == "P":
            pend = [int(f[1]), f[2], f[3], f[4]]
        elif f[0] == "Q":
            pend.append([int(x) for x in f[1:]])
        else:
            s = bytes(int(x, 16) for x in f[1:]).decode("utf-8")
            out["strings"].append({"player": pend[0], "p1": pend[1], "p2": pend[2],
                                   "legal": pend[3], "actions": pend[4], "text": s})
    for line in run("errors"):
        _, name, kind, *msg = line.split(" ")
        out["errors"][name] = {"kind": kind, "message": " ".join(msg)}
    (GOLD / "strings_errors.json").write_text(json.dumps(out, indent=1, ensure_ascii=False))
    print("strings:", len(out["strings"]), "errors:", len(out["errors"]))


def _real_features(n: int, history_size: int, seed: int) -> np.ndarray:
    """Feature planes of real positions (oracle restatement, pinned above;
    tests/ref_fixtures.py:real_features, which the GPU tests re-run)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    sys.path.insert(0, str(ROOT / "tests"))
    from ref_fixtures import real_features

    return real_features(n, history_size, seed)


def make_resnet() -> None:
    import torch

    sys.path.insert(0, str(REF_PY))
    from othello_alphazero.neural_net import AlphaZeroNet  # reference, read-only

    from othello_mcts.synthetic import alphazero_state_dict, net_config_from_state_dict

    torch.manual_seed(0)
    cases = {
        # name: (seed, H, C, blocks, hidden, n_boards)
        "tiny": (11, 8, 16, 2, 16, 32),
        "c128b9_h8": (1234, 8, 128, 9, 128, 16),
        "c128b9_h4": (4321, 4, 128, 9, 128, 8),
        "c256b19_h8": (2025, 8, 256, 19, 256, 4),
    }
    meta = {}
    arrays = {}
    for name, (seed, H, C, R, hid, n) in cases.items():
        sd = alphazero_state_dict(seed, 1 + 2 * H, C, R, hid)
        net = AlphaZeroNet(**net_config_from_state_dict(sd))
        net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
        net.eval()
        x = _real_features(n, H, seed)
        with torch.no_grad():
            out = net(torch.from_numpy(x))
        arrays[f"{name}_x"] = x.astype(np.int8)  # binary planes
        arrays[f"{name}_policy"] = out["policy"].numpy()
        arrays[f"{name}_value"] = out["value"].numpy()
        wsum = float(sum(np.asarray(v, np.float64).sum() for v in sd.values()))
        meta[name] = {"seed": seed, "history_size": H, "conv_channels": C,
                      "num_residual_blocks": R, "value_head_hidden_channels": hid,
                      "boards": n, "weight_sum": wsum}
        print("resnet", name, "policy row0 sum", float(out["policy"][0].sum()))
    np.savez_compressed(GOLD / "resnet.npz", **arrays)
    (GOLD / "resnet_meta.json").write_text(json.dumps(meta, indent=1))


def make_resnet_large() -> None:
    """The throughput geometries (>= 1024 rows per launch: 4-board C=128
    workgroups, the register-queue C=256 ones) against the reference's own
    AlphaZeroNet. Only (seed, rows) and a checksum of the planes are stored;
    tests/test_gpu_resnet.py regenerates the planes (ref_fixtures.real_features)."""
    import torch

    sys.path.insert(0, str(REF_PY))
    from othello_alphazero.neural_net import AlphaZeroNet  # reference, read-only

    from othello_mcts.synthetic import alphazero_state_dict, net_config_from_state_dict
    from ref_fixtures import planes_checksum

    torch.set_num_threads(8)
    cases = {
        # name: (weight seed, H, C, blocks, hidden, rows, planes seed); rows ragged
        # in the last workgroup (4 boards at C=128, 2 at C=256)
        "c128b9_h8_r1027": (1235, 8, 128, 9, 128, 1027, 71),
        "c128b9_h4_r1029": (4322, 4, 128, 9, 128, 1029, 72),
        "c256b19_h8_r1025": (2028, 8, 256, 19, 256, 1025, 73),
    }
    meta, arrays = {}, {}
    for name, (seed, H, C, R, hid, n, xseed) in cases.items():
        sd = alphazero_state_dict(seed, 1 + 2 * H, C, R, hid)
        net = AlphaZeroNet(**net_config_from_state_dict(sd))
        net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
        net.eval()
        x = _real_features(n, H, xseed)
        with torch.no_grad():
            out = net(torch.from_numpy(x))
        arrays[f"{name}_policy"] = out["policy"].numpy()
        arrays[f"{name}_value"] = out["value"].numpy()
        meta[name] = {"seed": seed, "history_size": H, "conv_channels": C, "num_residual_blocks": R,
                      "value_head_hidden_channels": hid, "boards": n, "planes_seed": xseed,
                      "planes_sha256_16": planes_checksum(x)}
        print("resnet large", name, "rows", n, "value[0]", float(out["value"][0]))
    np.savez_compressed(GOLD / "resnet_large.npz", **arrays)
    (GOLD / "resnet_large_meta.json").write_text(json.dumps(meta, indent=1))


def make_resnet_live() -> None:
    """The benched live nets (bench.py bench_state_dict: "live" for the headline
    and configs[3], "frontier" for the deep_tree record)
    against the reference's own AlphaZeroNet at throughput-geometry sizes. The
    weights are regenerated by the tests (synthetic.live_state_dict, float64
    calibration rounded to float32) and checked against the stored checksum;
    the planes likewise (ref_fixtures.real_features)."""
    import hashlib

    import torch

    sys.path.insert(0, str(REF_PY))
    from othello_alphazero.neural_net import AlphaZeroNet  # reference, read-only

    from othello_mcts.synthetic import live_state_dict, net_config_from_state_dict, selfplay_state_dict
    from ref_fixtures import planes_checksum

    torch.set_num_threads(8)
    cases = {
        # name: (policy, sharpness, weight seed, H, C, blocks, hidden, rows, planes seed); policy
        # "selfplay": the self-play trained net of bench_nets/ (the deep_tree record's)
        "selfplay_c128b9_h8_r1027": ("selfplay", 0.0, 0, 8, 128, 9, 128, 1027, 84),
        "live_c128b9_h8_r1027": ("random", 1.0, 2025, 8, 128, 9, 128, 1027, 81),
        "frontier_c128b9_h8_r1027": ("frontier", 1.25, 2025, 8, 128, 9, 128, 1027, 82),
        "live_c256b19_h8_r1025": ("random", 1.0, 2025, 8, 256, 19, 256, 1025, 83),
    }
    meta, arrays = {}, {}
    for name, (policy, sharp, seed, H, C, R, hid, n, xseed) in cases.items():
        sd = (selfplay_state_dict() if policy == "selfplay" else
              live_state_dict(seed, 1 + 2 * H, C, R, hid, policy=policy, policy_sharpness=sharp))
        h = hashlib.sha256()
        for k, v in sd.items():
            h.update(k.encode())
            h.update(np.ascontiguousarray(v).tobytes())
        net = AlphaZeroNet(**net_config_from_state_dict(sd))
        net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
        net.eval()
        x = _real_features(n, H, xseed)
        with torch.no_grad():
            out = net(torch.from_numpy(x))
        arrays[f"{name}_policy"] = out["policy"].numpy()
        arrays[f"{name}_value"] = out["value"].numpy()
        meta[name] = {"policy": policy, "policy_sharpness": sharp, "seed": seed, "history_size": H,
                      "conv_channels": C, "num_residual_blocks": R, "value_head_hidden_channels": hid,
                      "boards": n, "planes_seed": xseed, "planes_sha256_16": planes_checksum(x),
                      "weights_sha256_16": h.hexdigest()[:16],
                      "value_std": float(out["value"].std()), "mean_max_prior": float(out["policy"].max(1).values.mean())}
        print("resnet live", name, meta[name]["value_std"], meta[name]["mean_max_prior"])
    np.savez_compressed(GOLD / "resnet_live.npz", **arrays)
    (GOLD / "resnet_live_meta.json").write_text(json.dumps(meta, indent=1))


def make_mcts_known_answers() -> None:
    data = {
        "provenance": "SURVEY.md section 4 (measured with the compiled reference extension)",
        "cases": [
            {"name": "equivariant_h4_b16_s800", "stub": "equivariant", "history_size": 4,
             "num_threads": 1, "batch_size": 16, "num_simulations": 800,
             "dirichlet_epsilon": 0.0, "actions": [], "visit_counts": [145, 85, 288, 266]},
            {"name": "uniform_h3_b8_s64_after_19_18", "stub": "uniform", "history_size": 3,
             "num_threads": 1, "batch_size": 8, "num_simulations": 64,
             "dirichlet_epsilon": 0.0, "actions": [19, 18], "visit_counts": [14, 14, 14, 14]},
        ],
    }
    (GOLD / "mcts_known_answers.json").write_text(json.dumps(data, indent=1))


if __name__ == "__main__":
    if sys.argv[1:] == ["resnet_large"]:
        make_resnet_large()
        raise SystemExit(0)
    if sys.argv[1:] == ["resnet_live"]:
        make_resnet_live()
        raise SystemExit(0)
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "ref", "all"], check=True)
    make_bitboards()
    make_features()
    make_strings_errors()
    make_resnet()
    make_resnet_large()
    make_resnet_live()
    make_mcts_known_answers()

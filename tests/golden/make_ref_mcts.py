"""Generate the MCTS known-answer matrix and the ``_self_play`` fixture from the
COMPILED REFERENCE (run in the build container only; never on the GPU box).

The reference extension ``_othello_mcts_impl`` is built from
/root/reference/cpp/src/lib/{search_thread,mcts,othello_mcts}.cpp by
``make -C oracle mcts`` (oracle/Makefile) into oracle/_ref/. This script imports
that module (top-level name ``_othello_mcts_impl``; this repository's own
extension lives at ``othello_mcts._othello_mcts_impl`` and is never imported
here) and records, for every case of the matrix SURVEY.md §4 specifies
(num_threads=1, dirichlet_epsilon=0, equivariant and uniform stub nets,
batch_size in {1, 8, 16}, history_size in {4, 8}, fixed action sequences of
>= 10 moves, one of them through a pass), per move:

  * ``visit_counts()``         (mcts.cpp:45-52)
  * ``mean_action_values()``   (mcts.cpp:54-61), float32 bit patterns
  * ``self_play_data()``       (mcts.cpp:63-112): 8 feature tensors (binary,
    stored bit-packed) and 8 policy tensors (float32)
  * the root position after the search and the action then applied
    (mcts.cpp:114-165, tree reuse across the whole sequence).

It also runs the reference's own ``train._self_play`` (train.py:404-452) on the
compiled reference MCTS with a deterministic stub net and ``np.random.seed``:
per-move features / policies, the value sequence, and the actions the
reference's sampling rule chose (captured by a recording proxy around MCTS).

Usage:  python tests/golden/make_ref_mcts.py        (after make -C oracle mcts)
        python tests/golden/make_ref_mcts.py --endgame   (racy T=2 endgames only)
Outputs (committed): tests/golden/ref_mcts.json, ref_mcts.npz,
                     ref_self_play.json, ref_self_play.npz, ref_noise.*,
                     ref_mcts_endgame.json (--endgame)
Nothing from the reference (source, bytecode, binary) is copied into the repo.
"""

from __future__ import annotations

import json
import sys
import sysconfig
from pathlib import Path

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference

import numpy as np
import torch  # the reference's __init__.py imports torch before the extension

ROOT = Path(__file__).resolve().parents[2]
GOLD = ROOT / "tests" / "golden"
REF_SO = ROOT / "oracle" / "_ref" / ("_othello_mcts_impl" + sysconfig.get_config_var("EXT_SUFFIX"))
REF_PY = Path("/root/reference/python")

torch.set_num_threads(1)


def load_ref():
    if not REF_SO.exists():
        raise SystemExit(f"{REF_SO} missing: run `make -C oracle mcts` first")
    sys.path.insert(0, str(REF_SO.parent))
    import _othello_mcts_impl as om  # the compiled reference

    assert Path(om.__file__).resolve() == REF_SO.resolve(), om.__file__
    return om


# ---------------------------------------------------------------- stub nets
# SURVEY.md Appendix B.3; identical to oracle/oracle.py equivariant_stub /
# uniform_stub (torch fp32 on CPU), so the fixture and the tests feed the same
# numbers to the search.
def equivariant_stub(x: torch.Tensor) -> dict:
    x = x.to("cpu", torch.float32)
    C = x.shape[1]
    w = torch.linspace(-1, 1, C)
    sq = (x * w.view(1, C, 1, 1)).sum(dim=1).flatten(1)
    logits = torch.cat([sq, torch.full((x.shape[0], 1), -2.0)], dim=1)
    return {"policy": torch.softmax(logits, dim=1),
            "value": torch.tanh(sq.mean(dim=1) + 0.1 * x[:, 0].flatten(1).mean(dim=1))}


def uniform_stub(x: torch.Tensor) -> dict:
    n = x.shape[0]
    return {"policy": torch.full((n, 65), 1.0 / 65.0), "value": torch.zeros(n)}


STUBS = {"equivariant": equivariant_stub, "uniform": uniform_stub}


# ---------------------------------------------------------------- action sequences
def random_game(om, seed: int) -> list[int]:
    rng = np.random.default_rng(seed)
    p = om.Position.initial_position()
    acts = []
    while not p.is_terminal():
        la = p.legal_actions()
        a = int(la[rng.integers(len(la))])
        acts.append(a)
        p = p.apply_action(a)
    return acts


def game_with_pass(om) -> tuple[int, list[int], int]:
    """First seed whose random game passes at ply 14..50; returns (seed, actions, pass ply)."""
    for seed in range(1000):
        acts = random_game(om, seed)
        for i, a in enumerate(acts):
            if a == 64 and 14 <= i <= 50:
                return seed, acts, i
    raise RuntimeError("no game with a mid-game pass")


def pos_tuple(p) -> list:
    return [int(p.player()), f"{p.player1_discs():016x}", f"{p.player2_discs():016x}", f"{p.legal_moves():016x}"]


# ---------------------------------------------------------------- known-answer matrix
def _run_once(om, case: dict) -> dict:
    m = om.MCTS(history_size=case["history_size"], num_simulations=case["num_simulations"],
                num_threads=case["num_threads"], batch_size=case["batch_size"], dirichlet_epsilon=0.0)
    for a in case["prefix"]:
        m.apply_action(a)
    stub = STUBS[case["stub"]]
    rec = {"visits": [], "q": [], "feats": [], "pols": [], "roots": []}
    for a in case["actions"]:
        rec["roots"].append(pos_tuple(m.position()))
        m.search(stub)
        rec["visits"].append(m.visit_counts())
        rec["q"].append(np.array(m.mean_action_values(), np.float32))
        d = m.self_play_data()
        f = torch.stack(d["features"]).numpy()
        assert set(np.unique(f)) <= {0.0, 1.0}
        rec["feats"].append(np.packbits(f.astype(np.uint8).reshape(8, -1), axis=1))
        rec["pols"].append(torch.stack(d["policy"]).numpy().astype(np.float32))
        m.apply_action(a)
    return rec


def _key(rec: dict) -> tuple:
    return tuple(tuple(v) for v in rec["visits"]) + tuple(q.tobytes() for q in rec["q"])


def run_case(om, case: dict, arrays: dict) -> None:
    """num_threads = 1: one run (the reference is deterministic there). With
    more threads the reference's interleaving is racy: the case is run
    `repeats` times and the modal trajectory is recorded with its frequency."""
    runs = [_run_once(om, case) for _ in range(case.get("repeats", 1))]
    keys = [_key(r) for r in runs]
    modal = max(set(keys), key=keys.count)
    rec = runs[keys.index(modal)]
    if case.get("repeats", 1) > 1:
        case["modal_runs"] = keys.count(modal)
    case["root_positions"] = rec["roots"]
    case["num_children"] = [len(v) for v in rec["visits"]]
    name = case["name"]
    arrays[f"{name}__visits"] = np.concatenate([np.array(v, np.int32) for v in rec["visits"]])
    arrays[f"{name}__q_bits"] = np.concatenate(rec["q"]).view(np.uint32)
    arrays[f"{name}__features_packed"] = np.stack(rec["feats"])
    arrays[f"{name}__policy"] = np.stack(rec["pols"])
    extra = f" (modal {case['modal_runs']}/{case['repeats']})" if "modal_runs" in case else ""
    print(f"{name}: {len(rec['visits'])} moves, root visits move 0 {rec['visits'][0]}{extra}")


def make_matrix(om) -> None:
    seed, acts, pass_ply = game_with_pass(om)
    print(f"action sequence: seed {seed}, {len(acts)} plies, pass at ply {pass_ply}")
    win = lambda lo, n: (acts[:lo], acts[lo:lo + n])  # noqa: E731
    cases = []

    def add(name, stub, H, B, S, lo, n, T=1, repeats=1):
        prefix, seq = win(lo, n)
        cases.append({"name": name, "stub": stub, "history_size": H, "batch_size": B,
                      "num_threads": T, "num_simulations": S, "dirichlet_epsilon": 0.0,
                      "prefix": prefix, "actions": seq, "repeats": repeats})

    lo = max(0, pass_ply - 6)
    # the SURVEY sample (H=4, B=16, 800 sims from the initial position) and its continuation
    add("eq_h4_b16_s800_open", "equivariant", 4, 16, 800, 0, 12)
    add("eq_h8_b16_s800_pass", "equivariant", 8, 16, 800, lo, 12)
    add("eq_h4_b8_s200_pass", "equivariant", 4, 8, 200, lo, 14)
    add("eq_h8_b8_s200_open", "equivariant", 8, 8, 200, 0, 12)
    add("eq_h4_b1_s48_pass", "equivariant", 4, 1, 48, lo, 12)
    add("eq_h8_b1_s40_open", "equivariant", 8, 1, 40, 0, 10)
    add("uni_h4_b16_s320_pass", "uniform", 4, 16, 320, lo, 12)
    add("uni_h8_b16_s320_open", "uniform", 8, 16, 320, 0, 10)
    add("uni_h4_b8_s64_pass", "uniform", 4, 8, 64, lo, 12)
    add("uni_h8_b8_s96_mid", "uniform", 8, 8, 96, 20, 10)
    add("uni_h4_b1_s24_pass", "uniform", 4, 1, 24, lo, 12)
    add("uni_h8_b1_s32_open", "uniform", 8, 1, 32, 0, 10)
    # through to the end of the game: terminal leaves and the last plies
    add("eq_h4_b16_s160_end", "equivariant", 4, 16, 160, len(acts) - 12, 12)
    add("uni_h8_b8_s64_end", "uniform", 8, 8, 64, len(acts) - 10, 10)
    # several search threads: the reference's racy interleaving, modal trajectory
    # of repeated runs (the self-play default T=2 x B=16 at H=8 first)
    add("eq_h8_t2_b16_s800_open", "equivariant", 8, 16, 800, 0, 6, T=2, repeats=10)
    add("eq_h4_t2_b8_s160_pass", "equivariant", 4, 8, 160, lo, 10, T=2, repeats=10)
    add("uni_h4_t2_b16_s320_mid", "uniform", 4, 16, 320, 20, 8, T=2, repeats=10)
    add("eq_h4_t3_b4_s200_open", "equivariant", 4, 4, 200, 0, 8, T=3, repeats=10)
    add("eq_h4_t4_b8_s256_pass", "equivariant", 4, 8, 256, lo, 2, T=4, repeats=20)
    # the survey's root-batch quirk case (after actions 19, 18)
    cases.append({"name": "uni_h3_b8_s64_quirk", "stub": "uniform", "history_size": 3, "batch_size": 8,
                  "num_threads": 1, "num_simulations": 64, "dirichlet_epsilon": 0.0, "repeats": 1,
                  "prefix": [19, 18], "actions": acts[2:3] if acts[:2] == [19, 18] else [int(
                      om.Position.initial_position().apply_action(19).apply_action(18).legal_actions()[0])]})
    arrays: dict[str, np.ndarray] = {}
    for c in cases:
        run_case(om, c, arrays)
    meta = {"provenance": "compiled reference extension (oracle/Makefile target mcts), "
                          "tests/golden/make_ref_mcts.py",
            "torch": torch.__version__, "action_seed": seed, "pass_ply": pass_ply, "cases": cases}
    (GOLD / "ref_mcts.json").write_text(json.dumps(meta, indent=0))
    np.savez_compressed(GOLD / "ref_mcts.npz", **arrays)


# ---------------------------------------------------------------- _self_play fixture
class RecordingMCTS:
    """Proxy around the reference MCTS that records the actions _self_play applies."""

    def __init__(self, m):
        self._m = m
        self.applied: list[int] = []

    def apply_action(self, a):
        self.applied.append(int(a))
        return self._m.apply_action(a)

    def __getattr__(self, name):
        return getattr(self._m, name)


def make_self_play(om) -> None:
    sys.path.insert(0, str(REF_PY))
    import types
    from argparse import Namespace

    # train.py does `from othello_mcts import MCTS`: expose the compiled reference
    # module under that package name (what the reference's __init__.py re-exports)
    pkg = types.ModuleType("othello_mcts")
    for k in ("MCTS", "Position", "get_flips", "get_legal_moves"):
        setattr(pkg, k, getattr(om, k))
    sys.modules["othello_mcts"] = pkg
    from othello_alphazero import train  # reference, read-only

    params = dict(history_size=4, num_simulations=64, num_threads=1, batch_size=8, dirichlet_epsilon=0.0)
    out_meta = {"provenance": "reference train._self_play on the compiled reference MCTS", "games": []}
    arrays = {}
    for gi, np_seed in enumerate((20250222, 7)):
        m = RecordingMCTS(om.MCTS(**params))
        np.random.seed(np_seed)
        data = train._self_play(m, equivariant_stub, Namespace(self_play_temperature=1.0))
        f = torch.stack(data["features"]).numpy()
        assert set(np.unique(f)) <= {0.0, 1.0}
        n = f.shape[0]
        arrays[f"g{gi}__features_packed"] = np.packbits(f.astype(np.uint8).reshape(n, -1), axis=1)
        arrays[f"g{gi}__policy"] = torch.stack(data["policies"]).numpy().astype(np.float32)
        arrays[f"g{gi}__values"] = torch.stack(data["values"]).numpy().astype(np.float32)
        out_meta["games"].append({"np_seed": np_seed, "params": params, "temperature": 1.0,
                                  "temperature_moves": 12, "actions": m.applied,
                                  "samples": n, "feature_shape": list(f.shape[1:])})
        print(f"self_play game {gi}: {len(m.applied)} moves, {n} samples, first value {arrays[f'g{gi}__values'][0]}")
    (GOLD / "ref_self_play.json").write_text(json.dumps(out_meta, indent=0))
    np.savez_compressed(GOLD / "ref_self_play.npz", **arrays)


# ---------------------------------------------------------------- Dirichlet noise statistics
def make_noise_stats(om) -> None:
    """The reference's root visit counts under Dirichlet noise (nondeterministic:
    std::random_device-seeded mt19937, search_thread.cpp:22-24, :233), over
    many independent runs per setting: a distribution fixture (SURVEY.md §4
    'Stochastic parts')."""
    seed, acts, pass_ply = game_with_pass(om)
    settings = [
        {"name": "t1_b8_s64_h4_open", "prefix": [], "history_size": 4, "num_threads": 1, "batch_size": 8,
         "num_simulations": 64, "runs": 400},
        {"name": "t1_b8_s96_h4_mid", "prefix": acts[:20], "history_size": 4, "num_threads": 1, "batch_size": 8,
         "num_simulations": 96, "runs": 400},
        {"name": "t2_b16_s800_h8_open", "prefix": [], "history_size": 8, "num_threads": 2, "batch_size": 16,
         "num_simulations": 800, "runs": 200},
    ]
    arrays = {}
    for st in settings:
        rows = []
        for _ in range(st["runs"]):
            m = om.MCTS(history_size=st["history_size"], num_simulations=st["num_simulations"],
                        num_threads=st["num_threads"], batch_size=st["batch_size"], dirichlet_epsilon=0.25,
                        dirichlet_alpha=0.5)
            for a in st["prefix"]:
                m.apply_action(a)
            m.search(equivariant_stub)
            rows.append(m.visit_counts())
        v = np.array(rows, np.int32)
        arrays[st["name"]] = v
        print(f"noise {st['name']}: mean {v.mean(0).round(2)} std {v.std(0).round(2)}")
    (GOLD / "ref_noise.json").write_text(json.dumps({
        "provenance": "compiled reference, dirichlet_epsilon 0.25, alpha 0.5, equivariant stub; rows = runs",
        "settings": settings}, indent=0))
    np.savez_compressed(GOLD / "ref_noise.npz", **arrays)


# ---------------------------------------------------------------- racy endgames
def make_endgame_races(om, repeats: int = 20) -> None:
    """Several search threads at the END of a game, where whole batches of
    leaves are terminal. A thread whose batch is all terminal skips the NN
    round trip and backs up and selects again at once (search_thread.cpp:
    102-127), racing the other threads for the tree mutex, so repeated runs
    of the reference rarely agree (recorded: the distinct trajectories and how
    often each occurred). Every run's per-move visits and Q bits are stored,
    and the tests require the HIP search's trajectory to be one the reference
    produced. The last plies of the matrix's random game (through its pass),
    T = 2."""
    seed, acts, pass_ply = game_with_pass(om)
    cases = []
    for name, stub, H, B, S, n in (("eq_h4_t2_b8_s160_end", "equivariant", 4, 8, 160, 12),
                                   ("eq_h4_t2_b16_s320_end", "equivariant", 4, 16, 320, 12),
                                   ("uni_h4_t2_b8_s96_end", "uniform", 4, 8, 96, 10)):
        case = {"name": name, "stub": stub, "history_size": H, "batch_size": B, "num_threads": 2,
                "num_simulations": S, "dirichlet_epsilon": 0.0, "prefix": acts[:len(acts) - n],
                "actions": acts[len(acts) - n:], "repeats": repeats}
        runs = [_run_once(om, case) for _ in range(repeats)]
        keys = [_key(r) for r in runs]
        distinct = list(dict.fromkeys(keys))
        case["trajectories"] = [{"count": keys.count(k),
                                 "visits": [list(map(int, v)) for v in runs[keys.index(k)]["visits"]],
                                 "q_bits": [[int(x) for x in q.view(np.uint32)] for q in runs[keys.index(k)]["q"]]}
                                for k in distinct]
        case["trajectories"].sort(key=lambda t: -t["count"])
        cases.append(case)
        print(f"{name}: {len(distinct)} distinct trajectories in {repeats} runs, "
              f"counts {[t['count'] for t in case['trajectories']]}")
    (GOLD / "ref_mcts_endgame.json").write_text(json.dumps({
        "provenance": "compiled reference extension (oracle/Makefile target mcts), "
                      "tests/golden/make_ref_mcts.py --endgame", "torch": torch.__version__,
        "action_seed": seed, "cases": cases}, indent=0))


if __name__ == "__main__":
    om = load_ref()
    if "--endgame" in sys.argv:
        make_endgame_races(om)
    else:
        make_matrix(om)
        make_self_play(om)
        make_noise_stats(om)

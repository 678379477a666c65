"""Fixture for the search-level precision test:
tests/golden/search_dtype.{npz,json}.

What it holds, per net, for N mid-game positions:
  * the root visit counts of the fp32 search — the oracle's C restatement of
    the reference search (oracle/omcts_oracle.c, pinned by the compiled
    reference's fixtures) driving the fp32 AlphaZeroNet restatement
    (oracle/resnet_ref.py, pinned by the reference's own outputs) — i.e. what
    the reference's MCTS.search(AlphaZeroNet) computes: the leaf value of the
    module's fp32 forward feeds the backup directly (search_thread.cpp:130-190
    via othello_mcts.cpp:36-45, neural_net.py:138-172);
  * the same searches under a second random-stream key: the fp32 search's own
    spread when only the leaves' symmetry draws change (the reference draws
    them from std::random_device, search_thread.cpp:93-100, so two reference
    runs differ exactly this way).

Search: H = 8, T = 1 x B = 16, 800 simulations (50 batches), eps = 0
(no Dirichlet noise), c_base 20000, c_init 2.5. With eps = 0 and T = 1 a
search is a deterministic function of (position with its history, net, game
key). The key of game g under engine seed s is the engine's
(csrc/tree.hip reset: mix64(s ^ mix64(g + 0x632BE59BD9B4E019))); the GPU test
asserts the engine reports the same keys.

Positions: N games from the initial position, each played k = 12..40 plies by
sampling the self-play trained net's fp32 prior over the legal moves
(temperature 1, seeded); every final position has >= 2 legal moves. Stored as
action sequences (the engine replays them with apply_actions, so each root
carries its real history).

Nets: "selfplay" (bench_nets/selfplay_128x10b_h8, the trained net),
"live128" (the headline net, synthetic.live_state_dict seed 2025, 128x10b),
"live256" (configs[3]'s net, 256x20b, first N256 positions only: 8x the CPU
cost per evaluation).

Case "selfplay_t2": the trained net under the self-play settings the bench
runs (T = 2 x B = 16, eps = 0.25 Dirichlet noise drawn from the same key
streams, train.py:250's MCTS config), first N_T2 positions. The engine
computes the reference's thread interleaving deterministically (DESIGN.md
§2), so with the same key the only difference left is the NN precision;
under the other key the noise vectors differ too.

Runs in this container only (CPU; ~25 min with 8 threads). Imports nothing
from the reference. Usage: python tests/golden/make_search_dtype.py
[--only CASE ...] (recompute those cases, keep the others of the committed
fixture)
"""

from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
GOLD = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))
sys.path.insert(0, str(ROOT / "oracle"))

import torch  # noqa: E402

import oracle as O  # noqa: E402
import resnet_ref  # noqa: E402

H = 8
SIMS = 800
THREADS = 1
BATCH = 16
N = 128
N256 = 48
N_T2 = 64
SEEDS = (0x5EA4C4A1, 0x5EA4C4B2)  # engine seeds of key streams A and B
M64 = (1 << 64) - 1


def game_key(seed: int, g: int) -> int:
    """csrc/tree.hip reset: gs->key = mix64(seed ^ mix64(g + 0x632BE59BD9B4E019))."""
    lib = O.lib()
    return lib.orc_mix64((seed ^ lib.orc_mix64((g + 0x632BE59BD9B4E019) & M64)) & M64)


def nets() -> dict:
    """case -> (state_dict, positions, (num_threads, batch_size, dirichlet_epsilon))."""
    from othello_mcts.synthetic import live_state_dict, selfplay_state_dict

    base = (THREADS, BATCH, 0.0)
    return {"selfplay": (selfplay_state_dict(), N, base),
            "live128": (live_state_dict(2025, 17, 128, 9, 128), N, base),
            "live256": (live_state_dict(2025, 17, 256, 19, 256), N256, base),
            "selfplay_t2": (selfplay_state_dict(), N_T2, (2, 16, 0.25))}


def torch_sd(sd):
    return {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}


def make_positions(sd_trained) -> np.ndarray:
    """(N, 40) int32 action sequences, -1 padded."""
    rng = np.random.default_rng(20260218)
    sd = torch_sd(sd_trained)
    plies = 12 + (np.arange(N) * 7) % 29
    chains = [[O.initial_position()] for _ in range(N)]
    acts = [[] for _ in range(N)]
    for k in range(int(plies.max()) + 8):
        live = [g for g in range(N) if (len(acts[g]) < plies[g] or len(O.legal_actions(chains[g][-1])) < 2)
                and chains[g][-1].player != 0 and len(acts[g]) < 48]
        if not live:
            break
        x = np.stack([O.features(chains[g], H, 0) for g in live])
        with torch.no_grad():
            pol = resnet_ref.forward(sd, torch.from_numpy(x))["policy"].numpy().astype(np.float64)
        for i, g in enumerate(live):
            legal = O.legal_actions(chains[g][-1])
            p = pol[i, legal]
            p = p / p.sum() if p.sum() > 0 else np.full(len(legal), 1.0 / len(legal))
            a = int(legal[rng.choice(len(legal), p=p)])
            acts[g].append(a)
            chains[g].append(O.apply_action(chains[g][-1], a))
    out = np.full((N, 48), -1, np.int32)
    for g in range(N):
        last = chains[g][-1]
        assert last.player != 0 and len(O.legal_actions(last)) >= 2, g
        out[g, :len(acts[g])] = acts[g]
    return out


def replay(actions_row) -> list[int]:
    return [a for a in actions_row if a >= 0]


def search_all(sd, actions: np.ndarray, n: int, seed: int, params=(THREADS, BATCH, 0.0)) -> tuple[np.ndarray, np.ndarray]:
    """Root visit counts and Q (n, 65), indexed by action, fp32 oracle search."""
    threads, batch, eps = params
    sdt = torch_sd(sd)

    def nn(feat):
        with torch.no_grad():
            out = resnet_ref.forward(sdt, torch.from_numpy(np.ascontiguousarray(feat)))
        return out["policy"].numpy(), out["value"].numpy()

    visits = np.zeros((n, 65), np.int32)
    q = np.zeros((n, 65), np.float32)
    for g in range(n):
        m = O.OracleMCTS(history_size=H, num_simulations=SIMS, num_threads=threads, batch_size=batch,
                         dirichlet_epsilon=eps, game_key=game_key(seed, g))
        for a in replay(actions[g]):
            m.apply_action(int(a))
        sims = m.search(nn)
        L = threads * batch
        assert sims == L * ((SIMS + L - 1) // L)
        legal = O.legal_actions(m.position())
        visits[g, legal] = m.visit_counts()
        q[g, legal] = m.mean_action_values()
    return visits, q


def summary(va: np.ndarray, vb: np.ndarray) -> dict:
    pa = va / va.sum(1, keepdims=True)
    pb = vb / vb.sum(1, keepdims=True)
    tv = 0.5 * np.abs(pa - pb).sum(1)
    top = (va.argmax(1) == vb.argmax(1))
    return {"top_move_agreement": round(float(top.mean()), 4), "tv_mean": round(float(tv.mean()), 4),
            "tv_median": round(float(np.median(tv)), 4), "tv_max": round(float(tv.max()), 4)}


def main() -> None:
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    only = ap.parse_args().only
    torch.set_num_threads(8)
    allnets = nets()
    t0 = time.time()
    actions = make_positions(allnets["selfplay"][0])
    arrays = {"actions": actions}
    meta = {"history_size": H, "num_simulations": SIMS, "num_threads": THREADS, "batch_size": BATCH,
            "dirichlet_epsilon": 0.0, "c_puct_base": 20000.0, "c_puct_init": 2.5, "seeds": list(SEEDS),
            "positions": N, "plies": [int((r >= 0).sum()) for r in actions],
            "game_keys": {str(s): [str(game_key(s, g)) for g in range(N)] for s in SEEDS},
            "nets": {}, "generator": "tests/golden/make_search_dtype.py"}
    if only:  # keep the committed cases, recompute the named ones
        old = json.loads((GOLD / "search_dtype.json").read_text())
        old_arr = dict(np.load(GOLD / "search_dtype.npz", allow_pickle=False))
        assert np.array_equal(old_arr["actions"], actions)
        arrays.update(old_arr)
        meta["nets"].update(old["nets"])
    for name, (sd, n, params) in allnets.items():
        if only and name not in only:
            continue
        res = []
        for s in SEEDS:
            v, q = search_all(sd, actions, n, s, params)
            arrays[f"{name}_visits_{s:x}"] = v
            arrays[f"{name}_q_{s:x}"] = q
            res.append(v)
            print(f"{name} seed {s:x}: {time.time() - t0:.0f} s", flush=True)
        meta["nets"][name] = {"positions": n, "num_threads": params[0], "batch_size": params[1],
                              "dirichlet_epsilon": params[2], "fp32_key_a_vs_key_b": summary(*res)}
        print(name, meta["nets"][name], flush=True)
    np.savez_compressed(GOLD / "search_dtype.npz", **arrays)
    (GOLD / "search_dtype.json").write_text(json.dumps(meta, indent=1) + "\n")


if __name__ == "__main__":
    main()

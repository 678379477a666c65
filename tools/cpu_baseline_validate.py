"""Validate bench.py's cpu_baseline (the oracle port of the reference CPU path)
against the REFERENCE ITSELF, in this container only (it imports the compiled
reference extension from oracle/_ref and the reference's AlphaZeroNet from
/root/reference/python; never run on the GPU box).

configs[0]: 1 game from the initial position, 800 sims/move, T=2 x B=16,
history 8, dirichlet_epsilon 0.25, 128x10b fp32 on torch-CPU. For each torch
thread count (8, 4, 1) both legs play the same number of moves and report
simulations/s; the port must be within +-15% of the reference (BASELINE.md,
SURVEY.md §8(d): 1,705 / 1,295 / 491 sims/s at 8 / 4 / 1 cores, measured when
the survey was written).

Usage: python tools/cpu_baseline_validate.py [--moves 12]
Writes profiles/r03_cpu_baseline_validation.json.
"""

from __future__ import annotations

import argparse
import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SURVEY_ANCHOR = {8: 1705.0, 4: 1295.0, 1: 491.0}

REF_LEG = r"""
import sys, time, json, types
sys.dont_write_bytecode = True
import numpy as np, torch
torch.set_num_threads({threads})
sys.path.insert(0, "{ref_so_dir}")
import _othello_mcts_impl as om
sys.path.insert(0, "/root/reference/python")
pkg = types.ModuleType("othello_mcts"); pkg.MCTS = om.MCTS; sys.modules["othello_mcts"] = pkg
from othello_alphazero.neural_net import AlphaZeroNet
sys.path.insert(0, "{pkg_dir}")
from othello_mcts_synthetic import alphazero_state_dict, net_config_from_state_dict
sd = alphazero_state_dict(1, 17, 128, 9, 128)
net = AlphaZeroNet(**net_config_from_state_dict(sd))
net.load_state_dict({{k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}})
net.eval()
m = om.MCTS(history_size=8, num_simulations=800, num_threads=2, batch_size=16, dirichlet_epsilon=0.25)
sims = 0
with torch.no_grad():
    m.search(net)  # warm-up move (not timed)
    m.apply_action(m.position().legal_actions()[int(np.argmax(m.visit_counts()))])
    t0 = time.perf_counter()
    for _ in range({moves}):
        m.search(net)
        sims += 800
        m.apply_action(m.position().legal_actions()[int(np.argmax(m.visit_counts()))])
dt = time.perf_counter() - t0
print(json.dumps({{"sims": sims, "seconds": dt}}))
"""


def ref_leg(threads: int, moves: int) -> dict:
    # the synthetic-weights module of this repo, imported standalone (no
    # othello_mcts package import in the reference's process)
    syn_dir = Path("/tmp/oamd_validate")
    syn_dir.mkdir(exist_ok=True)
    (syn_dir / "othello_mcts_synthetic.py").write_text(
        (ROOT / "othello-alphazero_amd" / "othello_mcts" / "synthetic.py").read_text())
    code = REF_LEG.format(threads=threads, moves=moves, ref_so_dir=ROOT / "oracle" / "_ref", pkg_dir=syn_dir)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True,
                         env={"OMP_NUM_THREADS": str(threads), "PATH": "/usr/bin:/bin"})
    r = json.loads(out.stdout.strip().splitlines()[-1])
    return {"value": round(r["sims"] / r["seconds"], 1), "moves": moves, "seconds": round(r["seconds"], 2)}


def port_leg(threads: int, moves: int) -> dict:
    code = (
        "import sys, json, torch; sys.path.insert(0, %r); sys.path.insert(0, %r); "
        "torch.set_num_threads(%d); import bench; "
        "r = bench.cpu_baseline(8, 128, 9, 128, moves=%d, warmup_moves=1, threads=%d); print(json.dumps(r))"
    ) % (str(ROOT), str(ROOT / "othello-alphazero_amd"), threads, moves, threads)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True,
                         env={"OMP_NUM_THREADS": str(threads), "PATH": "/usr/bin:/bin"})
    r = json.loads(out.stdout.strip().splitlines()[-1])
    return {"value": r["value"], "sample": r["sample"], "cores": r["cores"]}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--moves", type=int, default=12)
    ap.add_argument("--threads", default="8,4,1")
    args = ap.parse_args()
    sys.path.insert(0, str(ROOT))
    import bench

    rows = []
    for t in [int(x) for x in args.threads.split(",")]:
        ref = ref_leg(t, args.moves)
        port = port_leg(t, args.moves)
        ratio = port["value"] / ref["value"]
        rows.append({"threads": t, "reference": ref, "port": port, "port_over_reference": round(ratio, 3),
                     "within_15pct": abs(ratio - 1.0) <= 0.15, "survey_anchor": SURVEY_ANCHOR.get(t)})
        print(json.dumps(rows[-1]), flush=True)
    out = {"what": "bench.py cpu_baseline (oracle port) vs the compiled reference, configs[0], same container",
           "cpu_model": bench.cpu_model(), "nproc": __import__("os").cpu_count(),
           "when": time.strftime("%Y-%m-%d %H:%M:%S"), "rows": rows}
    (ROOT / "profiles" / "r03_cpu_baseline_validation.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

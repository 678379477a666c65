"""Diagnostic: the drop-in MCTS (HIP, callback path) and the oracle with the
same game key, move by move over a racy-endgame fixture case
(tests/golden/ref_mcts_endgame.json): per-move visit counts of both and which
reference runs each follows. Test infrastructure (imports oracle/)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "othello-alphazero_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
import othello_mcts as om  # noqa: E402
import ref_fixtures as RF  # noqa: E402

for c in RF.load_endgame_cases():
    m = om.MCTS(history_size=c["history_size"], torch_device="cpu", num_simulations=c["num_simulations"],
                num_threads=2, batch_size=c["batch_size"], dirichlet_epsilon=0.0, seed=1234)
    m.set_native_nn(False)
    r = O.OracleMCTS(history_size=c["history_size"], num_simulations=c["num_simulations"], num_threads=2,
                     batch_size=c["batch_size"], dirichlet_epsilon=0.0, game_key=m.game_key())
    fn = O.equivariant_stub if c["stub"] == "equivariant" else O.uniform_stub

    def stub(f):
        p, v = fn(f.cpu().numpy())
        return {"policy": torch.from_numpy(p), "value": torch.from_numpy(v)}

    for a in c["prefix"]:
        m.apply_action(a)
        r.apply_action(a)
    for k, a in enumerate(c["actions"]):
        m.search(stub)
        r.search(fn)
        gv, ov = list(m.visit_counts()), list(r.visit_counts())
        gq = np.array(m.mean_action_values(), np.float32)
        oq = np.array(r.mean_action_values(), np.float32)
        print(c["name"], k, "visits equal" if gv == ov else f"VISITS DIFFER gpu {gv} oracle {ov}",
              "q max diff", float(np.abs(gq - oq).max()) if gv == ov else "-", flush=True)
        m.apply_action(a)
        r.apply_action(a)

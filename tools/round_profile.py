"""Diagnostic: where a self-play step's time goes between ResNet launches, from
a rocprofv3 kernel trace of bench.py (tools/gpu.sh `trace` recipe).

  python tools/round_profile.py gpurun_out/<run>/trace_<name>

Per pipeline group (stream), the k_tree launches are numbered by their round
within a search (a search = steps + 1 tree launches per group, the k_selfplay
move kernel ends it). Prints k_tree duration percentiles per round index, the
NN-idle time (no k_resnet running) attributed to what the next NN launch was
waiting for (its group's tree kernel still running, or nothing = dispatch
gap), and the share of the traced span with a k_resnet running.
"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np


def load(d: str):
    f = next(Path(d).glob("**/run_kernel_trace.csv"))
    rows = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Queue_Id"])))
    rows.sort()
    return rows


def main(d: str) -> None:
    rows = load(d)
    nn = [(s, e, q) for s, e, n, q in rows if "k_resnet" in n]
    tree = [(s, e, q) for s, e, n, q in rows if "k_tree" in n]
    moves = [(s, e, q) for s, e, n, q in rows if "k_selfplay" in n]
    # skip the warm-up: start at the first move kernel
    t0 = moves[0][1] if moves else rows[0][0]
    nn = [x for x in nn if x[0] > t0]
    tree = [x for x in tree if x[0] > t0]
    moves = [x for x in moves if x[0] > t0]
    span = (max(e for _, e, _ in nn) - t0) / 1e3
    busy = sum(e - s for s, e, _ in nn) / 1e3
    print(f"{len(nn)} k_resnet, {len(tree)} k_tree, {len(moves)} move kernels over {span / 1e3:.1f} ms; "
          f"k_resnet running {busy / span:.1%} of the span")
    # round index per tree launch: count per queue since that queue's last move boundary
    mv_ends = sorted(e for _, e, _ in moves)
    per_round = defaultdict(list)
    last_mv, ridx = {}, defaultdict(int)
    for s, e, q in tree:
        k = np.searchsorted(mv_ends, s)
        if last_mv.get(q) != k:
            last_mv[q] = k
            ridx[q] = 0
        per_round[ridx[q]].append((e - s) / 1e3)
        ridx[q] += 1
    print("k_tree duration by round (us): round n p50 p90 max")
    for r in sorted(per_round):
        v = np.array(per_round[r])
        print(f"  {r:3d} {len(v):6d} {np.median(v):8.1f} {np.percentile(v, 90):8.1f} {v.max():8.1f}")
    # NN idle gaps
    gaps_tree, gaps_other = 0.0, 0.0
    tree_by_q = defaultdict(list)
    for s, e, q in tree:
        tree_by_q[q].append((s, e))
    for (s0, e0, _), (s1, e1, q1) in zip(nn, nn[1:]):
        g = (s1 - e0) / 1e3
        if g <= 0:
            continue
        # the tree launch of the next NN's group that ended last before s1
        te = [e for s, e in tree_by_q[q1] if e <= s1]
        blocked = max(0.0, (te[-1] - e0) / 1e3) if te else 0.0
        blocked = min(blocked, g)
        gaps_tree += blocked
        gaps_other += g - blocked
    print(f"NN idle between launches: {gaps_tree + gaps_other:.0f} us total = {(gaps_tree + gaps_other) / span:.1%}; "
          f"waiting for the group's k_tree {gaps_tree:.0f} us, other (dispatch, move boundary) {gaps_other:.0f} us")
    d_nn = np.array([(e - s) / 1e3 for s, e, _ in nn])
    print(f"k_resnet duration us: p50 {np.median(d_nn):.1f} p10 {np.percentile(d_nn, 10):.1f} "
          f"p90 {np.percentile(d_nn, 90):.1f}")


if __name__ == "__main__":
    main(sys.argv[1])

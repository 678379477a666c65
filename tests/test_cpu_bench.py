"""bench.py's roofline arithmetic on a synthetic measurement (no GPU): the
achieved rate is the timed rounds' NN rows x FLOPs per row over the union of
their launch intervals, the round-2 basis divides by the
non-terminal share, and the tree timings split select rounds from the final
backup."""

import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def _m(launches=50, busy_per=0.75, span_per=1.05, rows=4096, evals_share=0.9, steps=10):
    return {"nn_ms": span_per * launches, "nn_busy_ms": busy_per * launches, "nn_launches": launches,
            "nn_rows": rows * launches, "timed_evals": int(rows * evals_share * launches),
            "select_ms": 0.45 * 25 * 2, "backup_ms": 0.13 * 2, "tree_launches": 25 * 2,
            "sims": 256 * 800 * steps, "evals": int(256 * 800 * steps * evals_share), "overflow_games": 0}


def test_roofline_uses_union_busy_time_and_timed_rows():
    args = bench.parse_args([])
    m = _m()
    out = bench.measured_fields(args, m, "w")
    r = out["roofline"]
    flops = bench.resnet_flops_per_eval(17, 128, 9, 128)
    n_eval = m["timed_evals"] / m["nn_launches"]
    expect = flops * n_eval / (0.75e-3) / 1e12
    assert r["achieved"] == pytest.approx(expect, rel=1e-4)
    assert r["frac"] == pytest.approx(expect / 2500.0, abs=1e-4)
    assert r["avg_launch_ms"] == pytest.approx(1.05) and r["busy_ms_per_launch"] == pytest.approx(0.75)
    # the round-2 basis counts every launched row: n_eval / the non-terminal share
    share = out["work"]["n_eval"] / out["work"]["rows_launched"]
    assert r["achieved_rows_launched"] == pytest.approx(r["achieved"] / share, rel=1e-3)
    assert out["work"]["terminal_share"] == pytest.approx(0.1, abs=1e-3)
    # tree: 25 select rounds per search and group, one final backup each
    t = out["tree_kernels"]
    assert t["k_tree"]["avg_launch_ms"] == pytest.approx(0.45)
    assert t["k_tree_final_backup"]["avg_launch_ms"] == pytest.approx(0.13)


def test_one_chain_union_equals_summed_durations():
    args = bench.parse_args(["--nn-chains", "1"])
    r = bench.measured_fields(args, _m(busy_per=0.8, span_per=0.8), "w")["roofline"]
    assert r["avg_launch_ms"] == r["busy_ms_per_launch"] and r["nn_chains"] == 1

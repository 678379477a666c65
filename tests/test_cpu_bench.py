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


def _m(launches=66, busy_per=0.75, span_per=1.05, rows=4096, evals_share=0.9, steps=10):
    # one sampled (HIP-event) search: 2 pipeline groups x 33 rounds (25 + 8
    # chain-splitting extra rounds); busy time and rows over every launch of
    # the window (steps searches)
    return {"nn_ms": span_per * launches, "nn_busy_ms": busy_per * launches * steps, "nn_launches": launches,
            "busy_launches": launches * steps, "nn_rows": rows * launches,
            "select_ms": 0.45 * 33 * 2, "backup_ms": 0.13 * 2, "tree_launches": 33 * 2, "final_launches": 2,
            "searches": steps, "rounds": 33 * steps,
            "sims": 256 * 800 * steps, "evals": int(256 * 800 * steps * evals_share), "overflow_games": 0,
            "depth_mean": 4.2, "depth_max_since_start": 17}


def test_roofline_uses_union_busy_time_and_timed_rows():
    args = bench.parse_args([])
    m = _m()
    out = bench.measured_fields(args, m, "w")
    r = out["roofline"]
    flops = bench.resnet_flops_per_eval(17, 128, 9, 128)
    n_eval = m["evals"] / m["busy_launches"]
    expect = flops * n_eval / (0.75e-3) / 1e12
    assert r["achieved"] == pytest.approx(expect, rel=1e-4)
    assert r["frac"] == pytest.approx(expect / 2500.0, abs=1e-4)
    assert r["avg_launch_ms"] == pytest.approx(1.05) and r["busy_ms_per_launch"] == pytest.approx(0.75)
    # the round-2 basis counts every launched row: n_eval / the non-terminal share
    share = out["work"]["n_eval"] / out["work"]["rows_launched"]
    assert r["achieved_rows_launched"] == pytest.approx(r["achieved"] / share, rel=1e-3)
    assert out["work"]["terminal_share"] == pytest.approx(0.1, abs=1e-3)
    assert out["work"]["depth_mean"] == 4.2 and out["work"]["depth_max_since_start"] == 17
    # tree: 33 select rounds per search and group (8 extra), one final backup each
    t = out["tree_kernels"]
    assert t["k_tree"]["avg_launch_ms"] == pytest.approx(0.45)
    assert t["k_tree_final_backup"]["avg_launch_ms"] == pytest.approx(0.13)
    assert t["rounds_per_search"] == 33 and t["max_rounds_per_search"] == 50


def test_one_chain_union_equals_summed_durations():
    args = bench.parse_args(["--nn-chains", "1"])
    r = bench.measured_fields(args, _m(busy_per=0.8, span_per=0.8), "w")["roofline"]
    assert r["avg_launch_ms"] == r["busy_ms_per_launch"] and r["nn_chains"] == 1


def test_rounds_per_search():
    """Every round of a search is an NN round: 25 batches per thread + up to
    chain_cuts extra rounds (exact interleaving only; the engine's adaptive
    count, reported as searches and rounds: the record carries the average);
    the timed region's k_resnet dispatches are the launches the engine saw."""
    a = bench.parse_args([])
    # 25 + min(64 cuts, 2 x 25 batches / budget 2)
    assert bench.max_search_rounds(a) == 50 and bench.pipeline_groups(a) == 2
    a = bench.parse_args(["--round-robin-endgames"])
    assert bench.max_search_rounds(a) == 25
    a = bench.parse_args(["--chain-budget", "0"])
    assert bench.max_search_rounds(a) == 25
    # configs[3]: 1600 sims = 50 batches per thread
    a = bench.parse_args(["--sims", "1600", "--channels", "256", "--blocks", "20"])
    assert bench.max_search_rounds(a) == 100
    # one game, T > 1: the thread-split schedule has no extra rounds
    a = bench.parse_args(["--games", "1"])
    assert bench.single_game_split(a) and bench.max_search_rounds(a) == 25
    # 10 searches averaging 28.5 rounds (25 + adaptive 3.5)
    m = _m()
    m.update(searches=10, rounds=285, busy_launches=570)
    out = bench.measured_fields(bench.parse_args([]), m, "w")
    assert out["tree_kernels"]["rounds_per_search"] == 28.5
    assert out["roofline"]["timed_region_launches"] == 570 == out["roofline"]["launches"]
    # no grouped search (the single-game split): the fixed count
    m.update(searches=0, rounds=0)
    out = bench.measured_fields(bench.parse_args(["--games", "1"]), m, "w")
    assert out["tree_kernels"]["rounds_per_search"] == 25


def test_n_eval_per_launch_within_launched_rows_with_extra_rounds():
    """With extra rounds present (near-empty launches for lagging games) the
    rows per launch still cover every launch of the timed searches: n_eval per
    launch <= rows per launch x (1 - terminal share)."""
    args = bench.parse_args(["--steps", "10"])
    # 10 searches: 10 x 2 x 33 launches of 4096-row capacity; the regular
    # rounds hold 0.9 of the rows as non-terminal, the extra rounds 2 %
    m = _m(launches=2 * 33)
    m["evals"] = int(10 * 2 * (25 * 4096 * 0.9 + 8 * 4096 * 0.02))
    m["sims"] = 256 * 800 * 10
    out = bench.measured_fields(args, m, "w")
    r = out["roofline"]
    share = out["work"]["terminal_share"]
    assert r["n_eval_per_launch"] <= r["rows_per_launch"] * (1 - share) + 1e-6
    assert r["timed_region_launches"] == 10 * 2 * 33
    assert len(r["kernel_hash"]) == 16


def _timing_lib(tmp_path):
    src = tmp_path / "u.cpp"
    src.write_text('''#include "timing.h"
#include <cstdio>
extern "C" double iu(const float* a, int n) {
    std::vector<std::pair<float, float>> v;
    for (int i = 0; i < n; ++i) v.emplace_back(a[2 * i], a[2 * i + 1]);
    return interval_union(v);
}
extern "C" double iu_ticks(const long long* a, int n) {
    std::vector<std::pair<long long, long long>> v;
    for (int i = 0; i < n; ++i) v.emplace_back(a[2 * i], a[2 * i + 1]);
    return interval_union(v);
}
''')
    so = tmp_path / "u.so"
    import subprocess

    subprocess.run(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-I", str(ROOT / "othello-alphazero_amd" / "csrc"),
                    str(src), "-o", str(so)], check=True)
    import ctypes

    lib = ctypes.CDLL(str(so))
    lib.iu.restype = ctypes.c_double
    lib.iu.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_int]

    def iu(pairs):
        import numpy as np

        a = np.ascontiguousarray(np.asarray(pairs, dtype=np.float32).reshape(-1))
        return lib.iu(a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(pairs))
    iu.lib = lib
    return iu


def test_interval_union_in_ticks_is_exact_over_long_windows(tmp_path):
    """the engine keeps the 100 MHz tick stamps as int64 through the
    union (float ms from the window start lost 0.01-0.06 ms per interval after
    minutes). One hour of 0.75 ms launches every 1 ms: exact."""
    import ctypes

    import numpy as np

    lib = _timing_lib(tmp_path).lib
    lib.iu_ticks.restype = ctypes.c_double
    lib.iu_ticks.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
    n = 3_600_000
    start = 10**12 + np.arange(n, dtype=np.int64) * 100_000  # 1 ms apart, ticks of 10 ns
    a = np.stack([start, start + 75_000], 1).reshape(-1)
    got = lib.iu_ticks(a.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), n)
    assert got == n * 75_000


def test_interval_union_of_the_engine(tmp_path):
    """csrc/timing.h: the busy time of overlapping NN chains. Intervals are
    measured from group 0's first event and another group's stream may run
    ahead of it (negative starts, more than 1 ms before): the union keeps them
    whole (a sweep anchored at 0 cut them)."""
    import random

    sys.path.insert(0, str(ROOT / "tools"))
    from prof_summary import interval_union as py_union

    iu = _timing_lib(tmp_path)
    assert iu([]) == 0.0
    assert iu([(-3.0, -2.0)]) == pytest.approx(1.0)
    assert iu([(-3.0, -1.5), (-2.0, 0.5), (1.0, 2.0)]) == pytest.approx(4.5)
    assert iu([(0.0, 4.0), (1.0, 2.0), (3.0, 5.0)]) == pytest.approx(5.0)
    rng = random.Random(3)
    for _ in range(200):
        xs = []
        for _ in range(rng.randint(1, 40)):
            a = rng.uniform(-20, 20)
            xs.append((a, a + rng.uniform(0, 3)))
        assert iu(xs) == pytest.approx(py_union(xs), abs=1e-4)


def test_sustained_record_uses_its_own_moves():
    """The `sustained` sub-record (moves after the timed region): its rate,
    rows launched and timed-region launches count its own moves."""
    args = bench.parse_args(["--steps", "10", "--sustained-moves", "64"])
    m = _m(steps=64)
    m["evals"] = int(m["sims"] * 0.85)
    out = bench.sustained_fields(args, m, 1, 800, 2.56)
    assert out["moves"] == 64 and out["value"] == pytest.approx(256 * 800 * 64 / 2.56, rel=1e-6)
    assert out["work"]["rows_launched"] == 256 * 800 * 64
    assert out["work"]["terminal_share"] == pytest.approx(0.15, abs=1e-3)
    assert out["roofline"]["timed_region_launches"] == 64 * 2 * 33


def test_byte_models():
    """Round 6: the tree kernels' algorithmic bytes are
    SURVEY §8(d)'s per-item constants over the engine's counters, per tree
    launch; the ResNet's are the weights once + 408 B per evaluated row; each
    line's counter traffic is divided by them."""
    args = bench.parse_args([])
    m = _m()
    tw = {"levels": 1000, "children_scanned": 9000, "expansions": 300, "children_created": 3000, "launches": 10}
    m["tree_work"] = tw
    out = bench.measured_fields(args, m, "w")
    t = out["tree_kernels"]["k_tree"]
    per_row = 8 * 16 + 17 * 8 + 65 * 2 + 2
    expect = 12 * 9000 + 32 * 1000 + 8 * 300 + 28 * 3000 + per_row * m["evals"]
    assert bench.tree_bytes_per_row(8) == per_row == 396
    assert t["algorithmic_bytes_per_launch"] == round(expect / 10)
    assert t["algorithmic_bytes_per_sim"] == pytest.approx(expect / m["sims"], abs=0.1)
    assert t["byte_model"]["children_scanned_per_level"] == 9.0
    assert t["byte_model"]["children_per_expansion"] == 10.0
    # 128x10b, H=8: 19 3x3 convs in bf16 (5.35 MB) + fp32 biases and heads
    wb = bench.resnet_weight_bytes(17, 128, 9, 128)
    convs = 9 * 17 * 128 + 18 * 9 * 128 * 128
    assert wb == 2 * convs + 4 * (19 * 128 + 387 + 8385 + 8320 + 129)
    r = out["roofline"]
    n_eval = m["evals"] / m["busy_launches"]
    assert r["algorithmic_bytes_per_launch"] == round(wb + 408 * n_eval)
    assert bench.RESNET_ROW_BYTES == 408


def test_host_budget():
    ranks = [{"rank": 0, "cpu_s_per_s": 0.08}, {"rank": 1, "cpu_s_per_s": 0.1}]
    h = bench.host_budget(ranks)
    assert h["ranks"] == 2 and h["cpu_s_per_s_max"] == 0.1 and h["cpu_s_per_s_sum"] == 0.18
    assert h["need_at_8_ranks"] == 0.8 and h["fits_8_ranks"] is (0.8 <= h["usable_cpus"])
    assert "cpu_s_per_s_max" not in bench.host_budget([{"rank": 0}])


def test_measured_ceiling_in_roofline():
    """The committed random-data MFMA ceiling (tools/mfma_ceiling.hip) is read
    into the roofline next to the spec-peak frac."""
    c = bench.mfma_ceiling("bf16")
    assert c is not None and 1000.0 < c["TFLOP_s"] <= 2500.0
    assert bench.mfma_ceiling("fp16") is not None and bench.mfma_ceiling("fp32") is None
    args = bench.parse_args([])
    r = bench.measured_fields(args, _m(), "w")["roofline"]
    mc = r["measured_ceiling"]
    assert mc["frac_achieved"] == pytest.approx(r["achieved"] / c["TFLOP_s"], abs=1e-3)
    assert mc["frac_executed"] == pytest.approx(r["executed_TFLOP_s"] / c["TFLOP_s"], abs=1e-3)
    assert r["frac"] == pytest.approx(r["achieved"] / 2500.0, abs=1e-4)  # the line's frac stays on the spec peak


def test_same_box_ceiling_parses_the_probe(tmp_path, monkeypatch):
    """same_box_ceiling runs tools/_build/mfma_ceiling with the dtypes' probe
    names and maps its JSON lines back to dtypes; with_ceiling puts the rate
    and both fractions into a roofline; a missing probe gives {}."""
    exe = tmp_path / "tools" / "_build" / "mfma_ceiling"
    exe.parent.mkdir(parents=True)
    exe.write_text("#!/bin/sh\n"
                   "echo \"args=$1\"\n"
                   "echo '{\"probe\": \"regs_random\", \"TFLOP_s\": 2000.0}'\n"
                   "echo '{\"probe\": \"f16_regs_random\", \"TFLOP_s\": 1900.0}'\n")
    exe.chmod(0o755)
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    assert bench.same_box_ceiling({"bf16", "fp16"}) == {"bf16": 2000.0, "fp16": 1900.0}
    assert bench.same_box_ceiling({"fp32"}) == {}
    r = {"achieved": 1800.0, "executed_TFLOP_s": 1650.0}
    bench.with_ceiling(r, 2000.0, "test")
    assert r["measured_ceiling"] == {"TFLOP_s": 2000.0, "source": "test", "frac_achieved": 0.9, "frac_executed": 0.825}
    exe.unlink()
    assert bench.same_box_ceiling({"bf16"}) == {}

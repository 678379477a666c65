"""Summarise rocprofv3 passes of tools/gpu.sh into profiles/ (build container).

  python tools/prof_summary.py nn OUTDIR PREFIX TAG
      the `nnpmc PREFIX_*` passes (standalone k_resnet launches of
      tools/nn_kernel.py) -> profiles/TAG_resnet_pmc.json
  python tools/prof_summary.py bench OUTDIR PREFIX TAG
      the `pmc PREFIX_*` passes over bench.py -> profiles/TAG_bench_pmc.json,
      and, with FETCH_SIZE + WRITE_SIZE passes, profiles/traffic_resnet.json
      (the bytes per launch bench.py reports as roofline.traffic)
  python tools/prof_summary.py trace OUTDIR NAME TAG
      `trace NAME` (kernel trace + stats) -> profiles/TAG_kernel_stats.csv

Per k_resnet dispatch (averaged over the dispatches of every pass):
  cycles       GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs)
  clock_GHz    cycles / kernel duration (MI355X_MICROARCH.md "DVFS give-back")
  mfma_busy    SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles)
  wave states  SQ_WAIT_ANY (parked: s_waitcnt / s_barrier), SQ_WAIT_INST_ANY
               (issue-stalled), SQ_ACTIVE_INST_ANY (issuing), / SQ_WAVE_CYCLES
  hbm_bytes    2 x FETCH_SIZE + WRITE_SIZE (KB -> B; gfx950 FETCH_SIZE counts
               half the bytes of a wide streaming read, MI355X_MICROARCH.md "HBM")
  l2_hit       TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
"""

import csv
import glob
import json
import re
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "profiles"
SIMDS = 256 * 4
FLOP_PER_CLK_SIMD = 1024  # dense bf16 / fp16: 16x16x32 MFMA (16 K FLOP) per 16 cycles


def flops_per_row(C: int, R: int, in_ch: int = 17, hidden: int | None = None) -> float:
    hidden = C if hidden is None else hidden
    return float(2 * 64 * 9 * in_ch * C + 2 * R * 2 * 64 * 9 * C * C + 2 * 64 * C * 3 + 2 * 128 * 65
                 + 2 * 64 * hidden + 2 * hidden)


def kernel_name_of(name: str) -> str:
    """k_resnet_w8<...> / k_tree(...) -> k_resnet_w8 / k_tree."""
    return re.split(r"[<(]", name.strip(), maxsplit=1)[0].split()[-1].split("::")[-1]


def gather(dirs: list[str], kernel: str = "k_resnet", regular_only: bool = True):
    """{counter: [per-dispatch values]} and [durations s] of the dispatches of
    `kernel` (a kernel-name prefix)."""
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    for d in dirs:
        for f in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if kernel_name_of(r["Kernel_Name"]).startswith(kernel):
                    per[(d, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for f in glob.glob(f"{d}/**/run_kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if kernel_name_of(r["Kernel_Name"]).startswith(kernel):
                    dur[(d, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    # per-launch counters of full launches: the chain-splitting extra rounds'
    # launches evaluate only lagging games' rows (mostly none) and are left out
    # of the per-launch averages (dispatches shorter than a quarter of the
    # median); the bench line's roofline covers every launch (trace_summary
    # cross-checks that)
    if dur and regular_only:
        med = sorted(dur.values())[len(dur) // 2]
        keep = {k for k, v in dur.items() if v >= 0.25 * med}
        dur = {k: v for k, v in dur.items() if k in keep}
        per = {k: v for k, v in per.items() if k in keep}
    by_counter = defaultdict(list)
    for key, cs in per.items():
        for c, v in cs.items():
            by_counter[c].append(v)
    return by_counter, list(dur.values())


def avg(xs):
    return sum(xs) / len(xs) if xs else None


def derive(c: dict, t: float | None, rows: int | None, fpr: float | None) -> dict:
    d = {}
    cyc = c.get("GRBM_GUI_ACTIVE")
    if cyc:
        cyc /= 8
        d["cycles_per_launch"] = round(cyc)
        if t:
            d["clock_GHz"] = round(cyc / t / 1e9, 3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            d["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc), 4)
        if "SQ_LDS_IDX_ACTIVE" in c:
            d["lds_array_busy_frac"] = round(c["SQ_LDS_IDX_ACTIVE"] / (256 * cyc), 4)
    w = c.get("SQ_WAVE_CYCLES")
    if w:
        for k, name in (("SQ_WAIT_ANY", "wave_parked_frac (s_waitcnt / s_barrier)"),
                        ("SQ_WAIT_INST_ANY", "wave_issue_stalled_frac"),
                        ("SQ_ACTIVE_INST_ANY", "wave_issuing_frac"),
                        ("SQ_WAIT_INST_LDS", "lds_issue_stall_frac")):
            if k in c:
                d[name] = round(c[k] / w, 4)
    m = c.get("SQ_INSTS_MFMA")
    if m:
        for k, name in (("SQ_INSTS_LDS", "lds_insts_per_mfma"), ("SQ_INSTS_SALU", "salu_insts_per_mfma"),
                        ("SQ_INSTS_VMEM", "vmem_insts_per_mfma")):
            if k in c:
                d[name] = round(c[k] / m, 3)
        if "SQ_INSTS_VALU" in c:
            d["non_mfma_valu_per_mfma"] = round(c["SQ_INSTS_VALU"] / m - 1, 3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            d["busy_cycles_per_mfma"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / m, 3)
    if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_bank_conflict_frac_of_lds_cycles"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        d["hbm_bytes_per_launch"] = round(2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024)
        if t:
            d["hbm_GB_s"] = round(d["hbm_bytes_per_launch"] / t / 1e9, 1)
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        d["l2_hit_frac"] = round(c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
    if t:
        d["avg_launch_ms"] = round(t * 1e3, 4)
        if rows and fpr:
            a = rows * fpr / t / 1e12
            d["achieved_TFLOP_s"] = round(a, 1)
            d["frac_of_2.5PF"] = round(a / 2500.0, 4)
            if "clock_GHz" in d:
                pk = SIMDS * FLOP_PER_CLK_SIMD * d["clock_GHz"] * 1e9 / 1e12
                d["frac_of_peak_at_held_clock"] = round(a / pk, 4)
    return d


def nn_summary(outdir: str, prefix: str, tag: str) -> dict:
    dirs = sorted(glob.glob(f"{outdir}/nnpmc_{prefix}_*"))
    dirs = [d for d in dirs if Path(d).is_dir()]
    by, durs = gather(dirs)
    c = {k: avg(v) for k, v in sorted(by.items())}
    line = ""
    for d in dirs:
        log = Path(d + ".log")
        if log.exists():
            for ln in log.read_text().splitlines():
                if ln.startswith("k_resnet "):
                    line = ln
    m = re.match(r"k_resnet (\d+)x(\d+)b (\w+)[^:]*: .*\(rows=(\d+)\)", line)
    rows = fpr = None
    if m:
        C, blocks, rows = int(m.group(1)), int(m.group(2)), int(m.group(4))
        fpr = flops_per_row(C, blocks - 1)
    res = {"tag": tag, "source": f"tools/gpu.sh nnpmc {prefix}_* over tools/nn_kernel.py ({line.strip()})",
           "passes": [Path(d).name for d in dirs], "dispatches_timed": len(durs),
           "counters_per_launch": {k: round(v) for k, v in c.items()},
           "derived": derive(c, avg(durs), rows, fpr)}
    OUT.mkdir(exist_ok=True)
    (OUT / f"{tag}_resnet_pmc.json").write_text(json.dumps(res, indent=1) + "\n")
    return res


def bench_summary(outdir: str, prefix: str, tag: str) -> dict:
    dirs = [d for d in sorted(glob.glob(f"{outdir}/pmc_{prefix}_*")) if Path(d).is_dir()]
    if not dirs:  # nothing to summarise: write nothing (the committed records stay)
        raise SystemExit(f"prof_summary: no PMC passes {outdir}/pmc_{prefix}_*")
    by, durs = gather(dirs)
    c = {k: avg(v) for k, v in sorted(by.items())}
    bench = None
    for d in dirs:
        log = Path(d + ".log")
        if log.exists():
            for ln in log.read_text().splitlines():
                if ln.startswith("{") and '"metric"' in ln:
                    bench = json.loads(ln)
    # the NN rows a regular launch evaluates (the per-launch counters above
    # skip the chain-splitting extra rounds' near-empty launches): the bench
    # line's n_eval over the regular rounds' launches (the extra rounds
    # evaluate lagging games only, none outside endgames)
    rows = None
    if bench:
        r, cfg = bench["roofline"], bench["config"]
        rounds = bench["tree_kernels"].get("rounds_per_search")
        regular = -(-cfg["sims_per_move"] // cfg["leaves_per_step"])
        launches = r.get("launches") or r.get("timed_region_launches")
        rows = (bench["work"]["n_eval"] / (launches * regular / rounds) if rounds and launches
                else r.get("n_eval_per_launch", r["rows_per_launch"]))
    if not bench:
        raise SystemExit(f"prof_summary: no bench line in the logs of {outdir}/pmc_{prefix}_*")
    fpr = bench["roofline"]["flops_per_row"]
    res = {"tag": tag, "source": f"tools/gpu.sh pmc {prefix}_* over bench.py",
           "workload": bench["config"]["workload"] if bench else None,
           "passes": [Path(d).name for d in dirs], "dispatches_timed": len(durs),
           "counters_per_launch": {k: round(v) for k, v in c.items()},
           "derived": derive(c, avg(durs), rows, fpr)}
    # k_tree over the same passes (every round: select rounds, extra rounds and
    # the final backups)
    tby, tdurs = gather(dirs, "k_tree", regular_only=False)
    tc = {k: avg(v) for k, v in sorted(tby.items())}
    res["k_tree"] = {"dispatches_timed": len(tdurs), "counters_per_launch": {k: round(v) for k, v in tc.items()},
                     "derived": derive(tc, avg(tdurs), None, None)}
    OUT.mkdir(exist_ok=True)
    (OUT / f"{tag}_bench_pmc.json").write_text(json.dumps(res, indent=1) + "\n")
    # the kernel sources these passes ran: the hashes the bench line read from
    # the library it loaded (not the sources on disk now)
    resnet_hash = bench["roofline"]["kernel_hash"]
    tree_hash = bench["tree_kernels"].get("kernel_hash")
    if tree_hash is None:  # bench lines before the tree hash was recorded
        sys.path.insert(0, str(ROOT))
        from bench import kernel_hash  # noqa: E402

        tree_hash = kernel_hash("tree")

    if "hbm_bytes_per_launch" in res["derived"]:
        (OUT / "traffic_resnet.json").write_text(json.dumps({
            "tag": tag, "bytes_per_launch": res["derived"]["hbm_bytes_per_launch"],
            "workload": bench["config"]["workload"], "rows_per_launch": bench["roofline"]["rows_per_launch"],
            "kernel_hash": resnet_hash,
            "note": "2 x FETCH_SIZE + WRITE_SIZE (KB -> B) per k_resnet launch, rocprofv3 --pmc, separate passes "
                    "(tools/prof_summary.py)"}, indent=1) + "\n")
    td = res["k_tree"]["derived"]
    if "hbm_bytes_per_launch" in td:
        (OUT / "traffic_tree.json").write_text(json.dumps({
            "tag": tag, "kernels": {"k_tree": {"bytes_per_launch": td["hbm_bytes_per_launch"],
                                               "avg_ms_rocprof": td.get("avg_launch_ms")}},
            "workload": bench["config"]["workload"], "kernel_hash": tree_hash,
            "note": "2 x FETCH_SIZE + WRITE_SIZE (KB -> B) per k_tree launch (every round of a search, final "
                    "backups included), rocprofv3 --pmc, separate passes (tools/prof_summary.py)"},
            indent=1) + "\n")
    return res


def trace_summary(outdir: str, name: str, tag: str) -> None:
    stats = next(Path(outdir).glob(f"trace_{name}/**/run_kernel_stats.csv"))
    OUT.mkdir(exist_ok=True)
    shutil.copy(stats, OUT / f"{tag}_kernel_stats.csv")
    trace = next(Path(outdir).glob(f"trace_{name}/**/run_kernel_trace.csv"), None)
    if trace is not None:
        res = resnet_busy(trace, bench_line(Path(outdir) / f"trace_{name}.log"))
        (OUT / f"{tag}_resnet_busy.json").write_text(json.dumps(res, indent=1) + "\n")
        print(json.dumps(res, indent=1))


def bench_line(log: Path) -> dict | None:
    if not log.exists():
        return None
    for ln in log.read_text().splitlines():
        if ln.startswith("{") and '"metric"' in ln:
            return json.loads(ln)
    return None


def interval_union(xs) -> float:
    """Length covered by [start, end] intervals (csrc/timing.h restated)."""
    xs = sorted(xs)
    busy, lo, hi = 0, None, None
    for a, b in xs:
        if hi is None or a > hi:
            if hi is not None:
                busy += hi - lo
            lo, hi = a, b
        else:
            hi = max(hi, b)
    return busy + (hi - lo if hi is not None else 0)


def resnet_busy(trace: Path, bench: dict | None = None) -> dict:
    """k_resnet dispatches of a kernel trace: mean duration, and the union of
    their [start, end] intervals per dispatch (launches of different NN chains
    overlap; bench.py's busy_ms_per_launch is the same union from HIP events).
    With the bench line of the traced command: the roofline recomputed from the
    trace alone — the timed region's rows (work.n_eval) x FLOPs per row over
    the union of its dispatches (the last roofline.timed_region_launches
    k_resnet dispatches: every round of every timed search) — next to the
    line's own frac."""
    iv = []
    with open(trace) as f:
        for row in csv.DictReader(f):
            if kernel_name_of(row["Kernel_Name"]).startswith("k_resnet"):
                iv.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    iv.sort()
    n = max(1, len(iv))
    res = {"source": str(trace), "dispatches": len(iv),
           "avg_duration_ms": round(sum(b - a for a, b in iv) / n / 1e6, 4),
           "busy_ms_per_dispatch": round(interval_union(iv) / n / 1e6, 4)}
    if not bench:
        return res
    # the dispatches run in this order: warm-up, the timed region, then the
    # `sustained` sub-record's moves (if any)
    segs = [("timed_region", bench, bench.get("roofline", {}))]
    if "sustained" in bench:
        segs.append(("sustained", bench["sustained"], bench["sustained"]["roofline"]))
    end = len(iv)
    for name, rec, r in reversed(segs):
        nt = r.get("timed_region_launches")
        if not nt or end < nt:
            break
        tr = iv[end - nt:end]
        end -= nt
        busy_ms = interval_union(tr) / 1e6
        n_eval = rec["work"]["n_eval"]
        fpr = bench["roofline"]["flops_per_row"]
        a = n_eval * fpr / (busy_ms * 1e-3) / 1e12
        res[name] = {"dispatches": nt,
                     "avg_duration_ms": round(sum(b - a_ for a_, b in tr) / nt / 1e6, 4),
                     "busy_ms_per_dispatch": round(busy_ms / nt, 4),
                     "n_eval": n_eval,
                     "trace_achieved_TFLOP_s": round(a, 1), "trace_frac": round(a / r["peak"], 4),
                     "bench_frac": r.get("frac"), "bench_busy_ms_per_launch": r.get("busy_ms_per_launch"),
                     "bench_n_eval_per_launch": r.get("n_eval_per_launch"),
                     "frac_rel_diff": round(r.get("frac", 0) / (a / r["peak"]) - 1, 4)}
    return res


if __name__ == "__main__":
    kind, outdir, prefix, tag = sys.argv[1:5]
    if kind == "nn":
        print(json.dumps(nn_summary(outdir, prefix, tag)["derived"], indent=1))
    elif kind == "bench":
        print(json.dumps(bench_summary(outdir, prefix, tag)["derived"], indent=1))
    else:
        trace_summary(outdir, prefix, tag)

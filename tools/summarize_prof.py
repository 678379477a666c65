"""Summarise rocprofv3 output (gpurun_out/prof) into profiles/<tag>_*.{csv,json}.

Per kernel: launches, average duration (kernel trace), FETCH_SIZE / WRITE_SIZE
per launch (KB; on gfx950 FETCH_SIZE counts 64 B per 128-B request, so read
bytes = 2 x FETCH_SIZE x 1024 for wide streaming reads, MI355X_MICROARCH.md
'HBM'), and any other PMC counters collected. Also writes
profiles/traffic_resnet.json (bytes per k_resnet launch) that bench.py reports.
"""

import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PROF = ROOT / "gpurun_out" / "prof"
OUT = ROOT / "profiles"


def main(tag: str) -> None:
    OUT.mkdir(exist_ok=True)
    stats = PROF / "trace" / "run_kernel_stats.csv"
    shutil.copy(stats, OUT / f"{tag}_kernel_stats.csv")
    pmc = defaultdict(lambda: defaultdict(list))
    for d in sorted(PROF.glob("pmc_*")):
        f = d / "run_counter_collection.csv"
        if not f.exists():
            continue
        for r in csv.DictReader(open(f)):
            pmc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kern = {}
    for r in csv.DictReader(open(stats)):
        kern[r["Name"]] = {"launches": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                           "pct": float(r["Percentage"])}
    for name, cs in pmc.items():
        k = kern.setdefault(name, {})
        for c, v in cs.items():
            k[c + "_per_launch"] = sum(v) / len(v)
    res = next((v for k, v in kern.items() if k.startswith("k_resnet")), {})
    # the bench line of the traced run names the workload the counters belong to
    bench_line = None
    log = PROF / "trace.log"
    if log.exists():
        for ln in log.read_text().splitlines():
            if ln.startswith("{") and '"metric"' in ln:
                bench_line = json.loads(ln)
    if "FETCH_SIZE_per_launch" in res and "WRITE_SIZE_per_launch" in res:
        fetch = 2.0 * res["FETCH_SIZE_per_launch"] * 1024  # gfx950 FETCH_SIZE correction
        write = res["WRITE_SIZE_per_launch"] * 1024
        res["hbm_bytes_per_launch"] = fetch + write
        (OUT / "traffic_resnet.json").write_text(json.dumps({
            "tag": tag, "bytes_per_launch": round(fetch + write),
            "fetch_bytes_corrected": round(fetch), "write_bytes": round(write),
            "workload": bench_line["config"]["workload"] if bench_line else None,
            "rows_per_launch": bench_line["roofline"]["rows_per_launch"] if bench_line else None,
            "note": "2 x FETCH_SIZE + WRITE_SIZE (KB -> B), rocprofv3 --pmc, separate passes"}, indent=1))
    tree = {}
    for name in ("k_tree",):
        k = kern.get(name, {})
        if "FETCH_SIZE_per_launch" in k and "WRITE_SIZE_per_launch" in k:
            tree[name] = {"bytes_per_launch": round(2.0 * k["FETCH_SIZE_per_launch"] * 1024
                                                    + k["WRITE_SIZE_per_launch"] * 1024),
                          "avg_ns_rocprof": k.get("avg_ns")}
    if tree:
        (OUT / "traffic_tree.json").write_text(json.dumps({
            "tag": tag, "kernels": tree,
            "workload": bench_line["config"]["workload"] if bench_line else None,
            "rows_per_launch": bench_line["roofline"]["rows_per_launch"] if bench_line else None,
            "note": "2 x FETCH_SIZE + WRITE_SIZE (KB -> B) per launch, rocprofv3 --pmc"}, indent=1))
    if "SQ_VALU_MFMA_BUSY_CYCLES_per_launch" in res and "GRBM_GUI_ACTIVE_per_launch" in res:
        # SQ_VALU_MFMA_BUSY_CYCLES sums MFMA-busy cycles over all SIMDs (1024 on MI355X);
        # GRBM_GUI_ACTIVE sums the GPU-active cycles over the 8 XCDs
        busy = res["SQ_VALU_MFMA_BUSY_CYCLES_per_launch"]
        active = res["GRBM_GUI_ACTIVE_per_launch"] / 8.0
        res["mfma_busy_frac"] = busy / (1024.0 * active) if active else None
    (OUT / f"{tag}_summary.json").write_text(json.dumps(kern, indent=1))
    print(json.dumps(kern, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")

"""Summarise a record set of tools/gpu.sh records (build container):
  python tools/record_summary.py gpurun_out/<N> <tag>
writes profiles/<tag>_<config>_kernel_stats.csv / _resnet_busy.json (trace
cross-checks) and prints the bench lines' headline, sustained and roofline
numbers next to the traces' own rooflines."""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
out, tag = Path(sys.argv[1]), sys.argv[2]


def line(f: Path):
    if not f.exists():
        return None
    ls = [json.loads(x) for x in f.read_text().splitlines() if x.startswith("{")]
    return ls[0] if ls else None


for n in ("c2", "s200", "c4", "c5"):
    if any(out.glob(f"trace_{n}/**/run_kernel_stats.csv")):
        subprocess.run([sys.executable, str(ROOT / "tools" / "prof_summary.py"), "trace", str(out), n, f"{tag}_{n}"],
                       check=True, capture_output=True)
for name in ("bench_c2", "launch_c2"):
    j = line(out / f"{name}.json")
    if j:
        s = j.get("sustained", {})
        print(name, j["value"], "frac", j["roofline"]["frac"], "| sustained", s.get("value"),
              s.get("roofline", {}).get("frac"), "| cpu", j.get("cpu_baseline", {}).get("value"),
              "| backend", j["config"]["backend"])
for n in ("c2", "s200", "c4", "c5"):
    f = ROOT / "profiles" / f"{tag}_{n}_resnet_busy.json"
    if f.exists():
        b = json.loads(f.read_text())
        for seg in ("timed_region", "sustained"):
            if seg in b:
                print(n, seg, {k: b[seg][k] for k in ("trace_frac", "bench_frac", "frac_rel_diff",
                                                      "busy_ms_per_dispatch", "bench_busy_ms_per_launch")})
t = out / "tests.log"
if t.exists():
    print([x for x in t.read_text().splitlines() if "passed" in x or "failed" in x][-1:])

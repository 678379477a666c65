"""Table of bench lines (value, frac, rounds per search, sustained) from the
bench_*.json files of a gpurun_out directory: python tools/ab_table.py DIR."""
import json
import sys
from pathlib import Path

for f in sorted(Path(sys.argv[1]).glob("bench*_*.json")):
    for ln in f.read_text().splitlines():
        if ln.startswith("{"):
            d = json.loads(ln)
            s = d.get("sustained", {})
            print(f"{f.stem.split('_', 1)[1]:14s} {d['value'] / 1e6:7.3f} M  frac {d['roofline']['frac']:.4f}  "
                  f"rounds {d['tree_kernels']['rounds_per_search']:7.3f} | sustained "
                  f"{s.get('value', 0) / 1e6:7.3f} M  frac {s.get('roofline', {}).get('frac', 0):.4f}  "
                  f"rounds {s.get('tree_kernels', {}).get('rounds_per_search', 0):7.3f}")

"""Gaps between consecutive k_resnet launches in a rocprofv3 kernel trace
(tools/gaps.py, bench.py): median / total gap and what runs inside the gaps."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 100
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40], r["Queue_Id"]) for r in rows)
nn = [k for k in ks if "k_resnet" in k[2]][-last:]
gaps = [nn[i + 1][0] - nn[i][1] for i in range(len(nn) - 1)]
gs = sorted(gaps)
print(f"k_resnet: {len(nn)} launches, mean {statistics.mean((k[1] - k[0]) / 1e3 for k in nn):.1f} us, "
      f"queues {sorted(set(k[3] for k in nn))}; gaps median {gs[len(gs) // 2] / 1e3:.1f} us, "
      f"sum {sum(gaps) / 1e3:.0f} us over a span of {(nn[-1][1] - nn[0][0]) / 1e3:.0f} us; "
      f"largest {[round(g / 1e3) for g in gs[-4:]]}")

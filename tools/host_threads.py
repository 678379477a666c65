"""Where a bench rank's host CPU time goes: run the
configs[1] workload's timed region (bench.py EngineWorkload, 20 steps after 5
warm-up) and print, per thread of this process, the CPU seconds it used over
the region (/proc/self/task/*/stat utime + stime) with the thread's name.
Usage (GPU box): python tools/host_threads.py [--spin-sync] [bench.py args]"""

import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402

TICK = os.sysconf("SC_CLK_TCK")


def threads() -> dict:
    out = {}
    for t in Path("/proc/self/task").iterdir():
        try:
            stat = (t / "stat").read_text()
            comm = (t / "comm").read_text().strip()
        except OSError:
            continue
        f = stat.rsplit(")", 1)[1].split()
        out[int(t.name)] = (comm, (int(f[11]) + int(f[12])) / TICK)
    return out


def main() -> None:
    args = bench.parse_args(["--steps", "20", "--warmup", "5"] + sys.argv[1:])
    wl = bench.EngineWorkload(args, 0, 0)
    wl.steps(args.warmup)
    wl.sync()
    t0 = threads()
    w0 = time.perf_counter()
    c0 = bench.cpu_seconds()
    wl.steps(args.steps)
    wl.sync()
    wall = time.perf_counter() - w0
    cpu = bench.cpu_seconds() - c0
    t1 = threads()
    rows = []
    for tid, (comm, c) in t1.items():
        d = c - t0.get(tid, (comm, 0.0))[1]
        if d > 0:
            rows.append({"tid": tid, "name": comm, "cpu_s": round(d, 3), "cpu_s_per_s": round(d / wall, 3)})
    rows.sort(key=lambda r: -r["cpu_s"])
    print(json.dumps({"wall_s": round(wall, 3), "cpu_s_per_s": round(cpu / wall, 3), "spin_sync": args.spin_sync,
                      "threads": rows[:12]}), flush=True)


if __name__ == "__main__":
    main()

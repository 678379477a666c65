"""Multi-process path of bench.py (section 5 of the task: games shard, no
data-path collective) on CPU with gloo, world_size 2, launched exactly like the
driver's N>1 run: python -m torch.distributed.run --master-addr 127.0.0.1."""

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gloo_bench_plumbing():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "tests" / "dist_worker.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints exactly one line
    out = json.loads(lines[0])
    assert out["world"] == 2
    shards = sorted(out["shards"], key=lambda s: s["rank"])
    assert [s["rank"] for s in shards] == [0, 1] and [s["local"] for s in shards] == [0, 1]
    # every rank saw the same max-over-ranks time, at least the slow rank's sleep
    assert shards[0]["dt_max"] == shards[1]["dt_max"] == out["dt_max"] >= 0.2
    # whole-job rate = all ranks' units / max time
    assert abs(out["rate"] - 2 * 2 * 32 / out["dt_max"]) < 1e-6 * out["rate"]
    # disjoint shards: distinct RNG keys and openings per rank, so different searches
    assert shards[0]["seeds"] != shards[1]["seeds"]
    assert shards[0]["played"] != shards[1]["played"]
    assert all(0 < sum(v) <= 32 for s in shards for v in s["played"])
    # the rank table names every rank's device and units (bench.py's n_gpus =
    # distinct devices, so ranks sharing a GPU are not counted twice)
    assert [r["rank"] for r in out["ranks"]] == [0, 1]
    assert len({r["device"] for r in out["ranks"]}) == 2 and all(r["sims"] == 64 for r in out["ranks"])


def test_single_rank_helpers():
    sys.path.insert(0, str(ROOT))
    import bench

    assert bench.shard_seeds(2025, 0) != bench.shard_seeds(2025, 1)
    assert bench.aggregate_rate(8, 256, 800, 10, 2.0) == 8 * 256 * 800 * 10 / 2.0
    calls = []
    dt = bench.timed_max(1, lambda: calls.append(1), lambda: calls.append(0), "cpu")
    assert calls == [0, 1, 0] and dt >= 0.0

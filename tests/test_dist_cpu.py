"""Multi-process path of bench.py (section 5 of the task: games shard, no
data-path collective) on the CPU: the real bench.main() rank path in --dry-run
mode (gloo, no GPU, each step a fixed sleep), launched both ways the driver
may start it — bare `bench.py --gpus 2`, which starts its own
torch.distributed.run child, and the driver's own `python -m
torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 bench.py
--gpus 2` — and the refusals: ranks != --gpus, and --gpus N without N GPUs."""

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
BENCH = str(ROOT / "bench.py")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env() -> dict:
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.pop("OAMD_BENCH_BACKEND", None)
    return env


def _run(cmd, timeout=300):
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=_env(), cwd=ROOT)


def _one_line(r) -> dict:
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints exactly one line
    return json.loads(lines[0])


def _check_line(out: dict, world: int, steps: int, step_ms: float, games: int) -> None:
    assert out["dry_run"] is True and "DRY RUN" in out["data"]
    assert out["metric"].startswith("MCTS simulations/sec (whole node)")
    assert out["n_gpus"] == world and out["steps"] == steps and out["scaling"] == "weak"
    ranks = sorted(out["config"]["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == list(range(world))
    assert len({r["device"] for r in ranks}) == world
    assert all(r["sims"] == games * 800 * steps for r in ranks)
    # per-rank time and rate: rank r sleeps (1 + r) x step_ms
    # per step. A rank's own time stops at its own final sync, before it waits
    # for the slower ranks at the closing barrier: rank 0 must NOT
    # read the slowest rank's time
    assert all(r["ms"] > 0 and abs(r["sims_per_s"] - r["sims"] / (r["ms"] / 1e3)) <= 1e-3 * r["sims_per_s"] + 0.1
               for r in ranks)
    for r in ranks:
        assert r["ms"] >= steps * (1 + r["rank"]) * step_ms
    assert ranks[0]["ms"] < 1.5 * steps * step_ms + 30.0
    assert ranks[-1]["ms"] > ranks[0]["ms"] + (world - 1) * steps * step_ms * 0.5
    # host budget: CPU seconds per wall second of each
    # rank's timed region; a sleeping dry-run rank uses almost none
    assert all(0.0 <= r["cpu_s_per_s"] < 0.5 for r in ranks)
    host = out["host"]
    assert host["ranks"] == world and host["usable_cpus"] >= 1
    assert host["cpu_s_per_s_max"] == max(r["cpu_s_per_s"] for r in ranks)
    assert host["need_at_8_ranks"] == round(8 * host["cpu_s_per_s_max"], 2)
    # the max over ranks: the last rank sleeps world x step_ms per step
    dt = out["ms_per_step"] * steps / 1e3
    assert dt >= steps * world * step_ms / 1e3
    assert dt * 1e3 >= max(r["ms"] for r in ranks)
    # whole-job rate = every rank's units / the max time
    assert abs(out["value"] - world * games * 800 * steps / dt) <= 1e-3 * out["value"] + 0.1
    assert "REHEARSAL" not in out["config"]["parallelism"] and out["config"]["backend"] == "gloo"
    assert "roofline" not in out
    # the CPU baseline rides on every world size's line (rank 0, after the
    # timed regions, the other ranks parked at a gloo barrier); a dry run
    # times one move of it
    cb = out["cpu_baseline"]
    assert cb["world_size"] == world and cb["moves"] == 1 and cb["value"] > 0 and cb["kind"] == "port"
    assert "dry run" in cb["note"]


def _check_two_rank_line(out: dict, steps: int, step_ms: float, games: int) -> None:
    _check_line(out, 2, steps, step_ms, games)


def test_bare_bench_gpus2_starts_its_own_ranks():
    r = _run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1",
              "--games", "4", "--dry-step-ms", "30"])
    assert "starting 2 ranks" in r.stderr
    _check_two_rank_line(_one_line(r), 3, 30.0, 4)


def test_driver_launch_gpus2():
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
              "--master-addr=127.0.0.1", f"--master-port={_free_port()}", BENCH,
              "--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "0", "--games", "8", "--dry-step-ms", "25"])
    assert "starting" not in r.stderr  # under a launcher bench.py starts nothing itself
    _check_two_rank_line(_one_line(r), 2, 25.0, 8)


def test_driver_launch_gpus8_dry_run():
    """the driver's N = 8 launch, rehearsed on the CPU: 8
    gloo ranks, the rank table, the MAX reduction (rank 7 is the slowest), the
    aggregate rate, the host budget and the CPU baseline at world size 8."""
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
              "--master-addr=127.0.0.1", f"--master-port={_free_port()}", BENCH,
              "--gpus", "8", "--dry-run", "--steps", "2", "--warmup", "0", "--games", "256", "--dry-step-ms", "15"],
             timeout=600)
    _check_line(_one_line(r), 8, 2, 15.0, 256)


def test_driver_launch_gpus1_joins_a_process_group():
    """Under a launcher even one rank runs the group path (on the GPU box: the
    RCCL init, barrier, MAX all-reduce and rank table of an N=1 run)."""
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
              "--master-addr=127.0.0.1", f"--master-port={_free_port()}", BENCH,
              "--gpus", "1", "--dry-run", "--steps", "2", "--warmup", "0", "--games", "4", "--dry-step-ms", "10"])
    out = _one_line(r)
    assert out["n_gpus"] == 1 and out["config"]["backend"] == "gloo"
    assert [x["rank"] for x in out["config"]["ranks"]] == [0]
    # a bare world-1 run has no process group
    out = _one_line(_run([sys.executable, BENCH, "--dry-run", "--steps", "1", "--warmup", "0", "--games", "4",
                          "--dry-step-ms", "5"]))
    assert out["config"]["backend"] == "none"


def test_ranks_must_match_gpus():
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
              "--master-addr=127.0.0.1", f"--master-port={_free_port()}", BENCH,
              "--gpus", "1", "--dry-run", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "--gpus 1 but the launcher started 2 rank(s)" in r.stdout + r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_gpus_without_gpus_fails_loudly():
    # this container has no GPU: a real (non-dry, non-rehearsal) 2-GPU run must
    # refuse before starting anything
    r = _run([sys.executable, BENCH, "--gpus", "2", "--steps", "1"], timeout=120)
    assert r.returncode != 0
    assert "needs 2 visible GPUs, found 0" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_single_rank_helpers():
    sys.path.insert(0, str(ROOT))
    import bench

    assert bench.shard_seeds(2025, 0) != bench.shard_seeds(2025, 1)
    assert bench.aggregate_rate(8, 256, 800, 10, 2.0) == 8 * 256 * 800 * 10 / 2.0
    calls = []
    dt, own, cpu = bench.timed_max(1, lambda: calls.append(1), lambda: calls.append(0), "cpu")
    assert calls == [0, 1, 0] and dt >= own >= 0.0 and cpu >= 0.0
    cpus = bench.usable_cpus()
    assert 1 <= cpus["usable"] <= cpus["nproc"]
    cmd = bench.launch_command(4, ["--gpus", "4"], 1234)
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-2:] == ["--gpus", "4"]
    # ranks sharing a device are refused outside the gloo rehearsal
    import pytest

    class A:
        gpus = 2
    shared = [{"rank": 0, "device": "h:u0", "sims": 1}, {"rank": 1, "device": "h:u0", "sims": 1}]
    with pytest.raises(SystemExit):
        bench.check_ranks(A, 2, "nccl", shared)
    bench.check_ranks(A, 2, "gloo", shared)  # the labelled rehearsal

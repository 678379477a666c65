import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "othello-alphazero_amd"
for p in (str(PKG), str(ROOT / "oracle"), str(ROOT), str(ROOT / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

os.environ.setdefault("OMP_NUM_THREADS", "4")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    import numerics

    if numerics.RECORDS:
        terminalreporter.section("numerics (max abs error vs fp32 yardsticks / Q ulp flips)")
        for case, text in numerics.RECORDS:
            terminalreporter.write_line(f"{case}: {text}")


@pytest.fixture(scope="session")
def golden_dir() -> Path:
    return ROOT / "tests" / "golden"


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False

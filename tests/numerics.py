"""Per-case numerical error records of the GPU tests (max |Δpolicy|, max
|Δvalue| of the native ResNet vs its fp32 yardsticks; Q ulp flips of the
search vs the reference). tests/conftest.py prints them in the pytest terminal
summary, so they land in the GPU test log tail."""

RECORDS: list[tuple[str, str]] = []


def record(case: str, text: str) -> None:
    RECORDS.append((case, text))

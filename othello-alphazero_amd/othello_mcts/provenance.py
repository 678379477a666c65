"""Source hashes of the native library.

build.py compiles these hashes into liboamd.so (`oamd_source_hash`), so a
caller can check that the library it loaded was built from the sources on
disk: `check_loaded_library()` raises when they differ (a stale prebuilt
library). The per-family hashes also key the committed PMC traffic records
(profiles/traffic_*.json, bench.py).
"""

from __future__ import annotations

import hashlib
from pathlib import Path

CSRC = Path(__file__).resolve().parent.parent / "csrc"
INCLUDE = Path(__file__).resolve().parent.parent.parent / "include"

# the sources each kernel family is compiled from
FAMILIES = {
    "resnet": ["resnet.hip", "kernels.h"],
    "tree": ["tree.hip", "engine.h", "bitboard.h", "rng.h", "kernels.h"],
    "all": ["bitboard.h", "capi.hip", "engine.h", "kernels.h", "resnet.hip", "rng.h", "timing.h", "tree.hip",
            "../../include/othello_mcts_amd.h", "../../include/othello_mcts_amd_experimental.h"],
}


def source_hash(kind: str) -> str:
    """sha256 (16 hex digits) over the sources of one family, as on disk."""
    h = hashlib.sha256()
    for name in FAMILIES[kind]:
        h.update(Path(name).name.encode())
        h.update((CSRC / name).read_bytes())
    return h.hexdigest()[:16]


def loaded_hash(kind: str) -> str:
    """The hash compiled into the loaded liboamd.so."""
    from ._othello_mcts_impl import source_hash as _lib_hash

    return _lib_hash(kind)


def check_loaded_library() -> dict:
    """{family: hash} of the loaded library; raises RuntimeError when any
    family differs from the sources on disk."""
    out = {}
    for kind in FAMILIES:
        lib, disk = loaded_hash(kind), source_hash(kind)
        if lib != disk:
            raise RuntimeError(f"liboamd.so was built from other sources than the ones on disk ({kind}: library "
                               f"{lib}, sources {disk}); rebuild with othello-alphazero_amd/build.py --force")
        out[kind] = lib
    return out

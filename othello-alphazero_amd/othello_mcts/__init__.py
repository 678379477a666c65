"""MI355X-native drop-in for the reference's ``othello_mcts`` package.

Same import surface as cpp/src/othello_mcts/__init__.py:1-6 (``MCTS``,
``Position``, ``get_flips``, ``get_legal_moves``), backed by hand-written HIP
kernels for gfx950 behind the C ABI in include/othello_mcts_amd.h. Additive
API: ``BatchedMCTS`` (G games per GPU, on-device self-play driver),
``NativeNet`` (fused bf16/fp16 AlphaZeroNet forward, also from a reference
checkpoint directory via ``load_checkpoint``), ``SelfPlayCollector`` /
``self_play`` (training samples in the reference's ``_self_play`` format) and
the training step beside the engine (``SampleBuffer``, ``train_epoch``,
``alphazero_loss``, ``refresh_native``: train.py:455-521 with the samples kept
in HBM).

There is no CPU fallback: importing works anywhere the extension was built,
but creating a search object needs a ROCm GPU and raises otherwise.
"""

# The reference imports torch first (its extension links libtorch). We keep the
# same order so user code that relies on it behaves identically.
import torch  # noqa: F401

from ._othello_mcts_impl import (  # noqa: F401
    MCTS,
    Position,
    SearchConfig,
    abi_version,
    device_count,
    get_flips,
    get_legal_moves,
)
from .batched import BatchedMCTS  # noqa: E402,F401
from .native import NativeNet, load_checkpoint  # noqa: E402,F401
from .selfplay import SelfPlayCollector, self_play  # noqa: E402,F401
from .training import SampleBuffer, alphazero_loss, refresh_native, train_epoch  # noqa: E402,F401

__all__ = [
    "MCTS",
    "Position",
    "get_flips",
    "get_legal_moves",
    "BatchedMCTS",
    "NativeNet",
    "SearchConfig",
    "SelfPlayCollector",
    "load_checkpoint",
    "self_play",
    "SampleBuffer",
    "alphazero_loss",
    "train_epoch",
    "refresh_native",
]

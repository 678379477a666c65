"""Native AlphaZeroNet evaluation (fused HIP kernel, csrc/resnet.hip).

``NativeNet`` packs a reference ``AlphaZeroNet`` state_dict
(python/othello_alphazero/neural_net.py:138-172; keys listed in SURVEY.md §5)
into the kernel's format: BatchNorm (eval, eps 1e-5) folded into each conv,
weights in MFMA fragment order, bf16 (default) or fp16. It is itself a valid
``NeuralNet`` callable (features -> {"policy", "value"}), and ``MCTS.search`` /
``BatchedMCTS.search`` recognise it and run the whole search on the GPU with
no Python in the loop.

``resolve`` is what ``MCTS.search`` calls on the object it is given: an
``AlphaZeroNet``-shaped module in eval mode (also behind ``torch.compile``) is
converted once and cached; the cache is invalidated whenever a parameter or
buffer is modified in place (tensor ``_version``), so a training loop that
updates the net between self-play games is always searched with fresh
weights. The switch from the module's fp32 forward to the native kernel's
fp16 (``MCTS(nn_dtype=...)``: "fp16" default, "bf16") is announced by a
one-time RuntimeWarning; only a module whose forward is the stock
AlphaZeroNet.forward is replaced. Set ``OTHELLO_MCTS_NATIVE_NN=0`` (or
``MCTS(native_nn=False)`` / ``set_native_nn(False)``) to always call the Python
module instead (the reference's exact numerics).

Why fp16 for the drop-in (round 6, tests/test_gpu_search_dtype.py, DESIGN.md
§9 "Search-level precision"): from 128 mid-game positions with the same
random streams, the native search's root visits are closer to the fp32
search's in fp16 than in bf16 on every net measured (trained 128x10b: mean
total-variation distance 0.084 vs 0.103, top move 0.86 vs 0.85; live
128x10b: 0.40 vs 0.51), and both are closer than the fp32 search is to itself
under another symmetry stream (0.19 trained). fp16's range is the risk:
``fp16_headroom`` measures the tower's largest activation on real positions
and a net without 16x headroom below the fp16 maximum is evaluated in bf16
(with a warning). The benchmark runs bf16 as BASELINE.json's configs[1]
states (NativeNet(dtype=...) is explicit there).
"""

from __future__ import annotations

import json
import os
import warnings
import weakref
from pathlib import Path

import numpy as np
import torch

from ._othello_mcts_impl import _Net
from .synthetic import net_config_from_state_dict

_DTYPES = {"bf16": 0, "bfloat16": 0, "fp16": 1, "float16": 1}
_DTYPES_NAME = {0: "bf16", 1: "fp16"}


def _to_numpy_state(sd) -> dict[str, np.ndarray]:
    out = {}
    for k, v in sd.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().to("cpu", torch.float32).numpy()
        out[k] = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
    return out


def load_checkpoint(checkpoint_dir) -> tuple[dict, dict]:
    """Read a reference checkpoint directory: ``config.json`` + ``neural_net.pth``
    as written by train.py:299-313 and read by player.py:195-228 (same
    in_channels validation and messages). The state_dict is loaded with
    ``weights_only=True`` on the CPU. Returns (config, state_dict); the
    ``config["neural_net"]`` entries must agree with the state_dict's shapes."""
    checkpoint_dir = Path(checkpoint_dir)
    with (checkpoint_dir / "config.json").open(encoding="utf-8") as f:
        config = json.load(f)
    in_channels = config["neural_net"]["in_channels"]
    if in_channels % 2 != 1:
        raise ValueError(f"Expected in_channels to be odd, but got {in_channels}.")
    history_size = (in_channels - 1) // 2
    if history_size < 1:
        raise ValueError(f"Expected history_size to be positive, but got {history_size}.")
    sd = torch.load(checkpoint_dir / "neural_net.pth", map_location="cpu", weights_only=True)
    got = net_config_from_state_dict(sd)
    for k, v in config["neural_net"].items():
        if k in got and got[k] != v:
            raise ValueError(f"config.json neural_net.{k} = {v} but neural_net.pth has {got[k]}")
    return config, sd


class NativeNet:
    """Fused-kernel AlphaZeroNet on one GPU (eval mode only)."""

    @classmethod
    def from_checkpoint(cls, checkpoint_dir, device: int | str | torch.device | None = None,
                        dtype: str = "bf16") -> "NativeNet":
        """NativeNet from a reference checkpoint directory (load_checkpoint)."""
        _, sd = load_checkpoint(checkpoint_dir)
        return cls(sd, device=device, dtype=dtype)

    def __init__(self, net_or_state_dict, device: int | str | torch.device | None = None,
                 dtype: str = "bf16") -> None:
        if hasattr(net_or_state_dict, "state_dict"):
            mod = getattr(net_or_state_dict, "_orig_mod", net_or_state_dict)
            sd = mod.state_dict()
        else:
            sd = net_or_state_dict
        self.config = net_config_from_state_dict(sd)
        if dtype not in _DTYPES:
            raise ValueError(f"dtype must be one of {sorted(_DTYPES)}, got {dtype!r}")
        self.dtype = dtype
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device if isinstance(device, int) else torch.device(device).index or 0)
        c = self.config
        self._net = _Net(self.device.index, c["in_channels"], c["conv_channels"], c["num_residual_blocks"],
                         c["value_head_hidden_channels"], _DTYPES[dtype])
        self.load_state_dict(sd)

    def load_state_dict(self, sd) -> None:
        arrs = _to_numpy_state(sd)
        tensors = []
        for key, numel in self._net.state_keys():
            a = arrs[key].reshape(-1)
            if a.size != numel:
                raise ValueError(f"{key}: expected {numel} elements, got {a.size}")
            tensors.append(a)
        self._net.load_state(tensors)

    @property
    def handle(self) -> int:
        return self._net.handle

    @property
    def history_size(self) -> int:
        return (self.config["in_channels"] - 1) // 2

    def __call__(self, features: torch.Tensor) -> dict[str, torch.Tensor]:
        x = features.to(self.device, torch.float32).contiguous()
        rows = x.shape[0]
        policy = torch.empty((rows, 65), dtype=torch.float32, device=self.device)
        value = torch.empty((rows,), dtype=torch.float32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        self._net.forward(x.data_ptr(), rows, policy.data_ptr(), value.data_ptr(), stream)
        return {"policy": policy, "value": value}


FP16_MAX = 65504.0
FP16_HEADROOM = 16.0


@torch.no_grad()
def fp16_headroom(sd, history_size: int, positions: int = 32, device="cpu") -> float:
    """FP16_MAX / the largest |activation| the kernel stores between layers
    (every conv's BN-folded output, before and after ReLU, and every residual
    sum), over the fp32 eval-mode forward (neural_net.py:9-128) of `positions`
    real positions (synthetic.calibration_features). > FP16_HEADROOM: fp16 is
    safe for this net."""
    import torch.nn.functional as F

    from .synthetic import calibration_features

    t = {k: torch.as_tensor(np.asarray(v, np.float32) if not isinstance(v, torch.Tensor) else v)
         .to(device=device, dtype=torch.float32) for k, v in sd.items() if not k.endswith("num_batches_tracked")}
    x = torch.from_numpy(calibration_features(positions, history_size, 11)).to(device)
    peak = 0.0

    def bn(h, p):
        return F.batch_norm(h, t[p + ".running_mean"], t[p + ".running_var"], t[p + ".weight"], t[p + ".bias"],
                            training=False, eps=1e-5)

    def conv(h, p, norm, pad=1):
        nonlocal peak
        y = bn(F.conv2d(h, t[p + ".weight"], t[p + ".bias"], padding=pad), norm)
        peak = max(peak, float(y.abs().max()))
        return y

    h = F.relu(conv(x, "conv_block.conv", "conv_block.norm"))
    i = 0
    while f"residual_blocks.{i}.conv1.weight" in t:
        p = f"residual_blocks.{i}"
        a = F.relu(conv(h, p + ".conv1", p + ".norm1"))
        h = conv(a, p + ".conv2", p + ".norm2") + h
        peak = max(peak, float(h.abs().max()))
        h = F.relu(h)
        i += 1
    conv(h, "policy_head.conv", "policy_head.norm", 0)
    conv(h, "value_head.conv", "value_head.norm", 0)
    return FP16_MAX / max(peak, 1e-30) if np.isfinite(peak) else 0.0


def _looks_like_alphazero(m) -> bool:
    """An AlphaZeroNet (neural_net.py:138-172) whose forward is the stock one: a
    subclass that overrides forward (logits, temperature, ...) is never
    replaced by the native kernel, which computes the stock forward."""
    if not all(hasattr(m, a) for a in ("conv_block", "residual_blocks", "policy_head", "value_head")):
        return False
    for cls in type(m).__mro__:
        if "forward" in vars(cls):
            return cls.__name__ == "AlphaZeroNet"
    return False


_warned: set = set()


def _warn_once(m, dtype: str, note: str = "") -> None:
    key = (id(type(m)), dtype, note)
    if key in _warned:
        return
    _warned.add(key)
    warnings.warn(
        f"othello_mcts: evaluating {type(m).__name__} with the native fused kernel in {dtype} "
        "(the reference calls the module's own fp32 forward); near-tied visit counts can differ "
        "(DESIGN.md §9: from the same positions and random streams the fp16 search picks the fp32 search's "
        "move in ~86 % of positions, the fp32 search itself in ~71 % under another symmetry stream). "
        "MCTS(..., native_nn=False) / set_native_nn(False) or OTHELLO_MCTS_NATIVE_NN=0 keeps the "
        "module's forward." + note,
        RuntimeWarning, stacklevel=3)


_cache: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def _signature(m) -> tuple:
    sig = []
    for t in list(m.parameters()) + list(m.buffers()):
        sig.append((t.data_ptr(), t._version))
    return tuple(sig)


def resolve(neural_net, device: int, history_size: int, dtype: str = "fp16"):
    """NativeNet to use for ``neural_net`` on ``device``, or None (call it instead).

    A NativeNet is used as given. A stock AlphaZeroNet module in eval mode is
    converted once to a NativeNet of ``dtype`` (cached until a parameter or
    buffer changes) and a one-time RuntimeWarning names the precision switch.
    fp16 is used only for a net with FP16_HEADROOM below the fp16 maximum
    (fp16_headroom); otherwise bf16, and the warning says so."""
    if isinstance(neural_net, NativeNet):
        if neural_net.device.index != device:
            raise ValueError(f"NativeNet lives on cuda:{neural_net.device.index}, the search on cuda:{device}")
        if neural_net.history_size != history_size:
            raise ValueError("NativeNet in_channels does not match 1 + 2 * history_size")
        return neural_net
    if os.environ.get("OTHELLO_MCTS_NATIVE_NN", "1") == "0":
        return None
    if dtype not in _DTYPES:
        raise ValueError(f"nn_dtype must be one of {sorted(_DTYPES)}, got {dtype!r}")
    m = getattr(neural_net, "_orig_mod", neural_net)
    if not isinstance(m, torch.nn.Module) or not _looks_like_alphazero(m) or m.training:
        return None
    try:
        cfg = net_config_from_state_dict(m.state_dict())
    except (KeyError, AttributeError):
        return None
    if cfg["conv_channels"] not in (128, 256) or cfg["in_channels"] != 1 + 2 * history_size:
        return None
    if cfg["num_squares"] != 64 or cfg["num_actions"] != 65:
        return None
    sig = _signature(m)
    hit = _cache.get(m)
    if hit is not None and hit[0] == sig and hit[1].device.index == device and hit[2] == dtype:
        return hit[1]
    use, note = _DTYPES_NAME[_DTYPES[dtype]], ""
    if use == "fp16":
        room = fp16_headroom(m.state_dict(), history_size, device=torch.device("cuda", device))
        if room < FP16_HEADROOM:
            use = "bf16"
            note = (f" fp16 was requested, but the net's largest activation on real positions leaves only "
                    f"{room:.1f}x headroom below the fp16 maximum (< {FP16_HEADROOM:g}x): bf16 is used.")
    _warn_once(m, use, note)
    nn_ = NativeNet(m, device=device, dtype=use)
    _cache[m] = (sig, nn_, dtype)
    return nn_

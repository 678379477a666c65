"""Winograd F(2x2, 3x3) tower probe vs the direct tower.

A measurement, not product code. Builds nothing: tools/_build/libwinoprobe*.so
are compiled in the build container (hipcc, see tools/winograd_probe.hip).

1. Correctness: two layers (a residual block: conv + bias + ReLU, conv + bias
   + skip + ReLU) on 5 boards against torch fp32 convolutions of the same
   bf16-rounded inputs (the probe rounds U = G g G^T, V = B^T d B and the
   activations to bf16).
2. Timing: 4096 boards (the headline's launch size), 18 layers (the 9
   residual blocks of 128x10b), median of 5 x 10 launches, against
   NativeNet (csrc/resnet.hip k_resnet_w8, the whole 19-conv forward with
   heads) on 4096 rows, same process, interleaved.
Prints one JSON line per library variant.
Usage (GPU box): python tools/winograd_probe.py [lib.so ...]
"""

import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))
sys.path.insert(0, str(ROOT))

G = np.array([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], np.float64)


def bf16_round(a: torch.Tensor) -> torch.Tensor:
    return a.to(torch.bfloat16).to(torch.float32)


def pack_u(ws: list[np.ndarray], q: int) -> torch.Tensor:
    """Per layer W (128, 128, 3, 3) -> U = G g G^T (16 points), bf16, in the
    probe's fragment order [layer][cb][xi][ob][lane][8] + q zero fragments."""
    frags = []
    lane = np.arange(64)
    for w in ws:
        gw = np.einsum("ai,ocij,bj->ocab", G, w.astype(np.float64), G)  # (out, in, 4, 4)
        U = gw.reshape(128, 128, 16)  # xi = 4a + b
        L = np.empty((4, 16, 8, 64, 8), np.float32)
        for cb in range(4):
            for ob in range(8):
                out = ob * 16 + (lane & 15)
                ins = cb * 32 + (lane >> 4)[:, None] * 8 + np.arange(8)[None, :]
                L[cb, :, ob] = U[out[:, None], ins, :].transpose(2, 0, 1)
        frags.append(L.reshape(-1))
    frags.append(np.zeros(q * 8 * 64 * 8, np.float32))
    t = torch.from_numpy(np.concatenate(frags)).to(torch.bfloat16)
    return t.view(torch.int16)


def reference(x, ws, bs):
    """fp32 torch: x (N, 64, 128) channel-last bf16 values -> the probe's layers."""
    h = x.view(-1, 8, 8, 128).permute(0, 3, 1, 2).float()
    skip = None
    for i, (w, b) in enumerate(zip(ws, bs)):
        if i % 2 == 0:
            skip = h
        y = F.conv2d(h, torch.from_numpy(w), torch.from_numpy(b), padding=1)
        if i % 2 == 1:
            y = y + skip
        h = bf16_round(F.relu(y))
    return h.permute(0, 2, 3, 1).reshape(x.shape)


def run(lib, x, U, bias, boards, layers, out):
    s = torch.cuda.current_stream().cuda_stream
    rc = lib.wino_probe_launch(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(U.data_ptr()),
                               ctypes.c_void_p(bias.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                               boards, layers, ctypes.c_void_p(s))
    assert rc == 0


def timed(fn, reps=10, outer=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(outer):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b) / reps)
    ms.sort()
    return ms[len(ms) // 2]


def main() -> None:
    libs = sys.argv[1:] or [str(ROOT / "tools" / "_build" / "libwinoprobe.so")]
    rng = np.random.default_rng(3)
    dev = torch.device("cuda", 0)
    # direct kernel: the headline's 128x10b forward on 4096 rows
    import bench
    import othello_mcts as om
    from othello_mcts.synthetic import calibration_features

    sd = bench.bench_state_dict("live", 2025, 17, 128, 9, 128)
    net = om.NativeNet(sd, device=0, dtype="bf16")
    xin = torch.from_numpy(calibration_features(4096, 8, 7)).to(dev)
    for path in libs:
        lib = ctypes.CDLL(path)
        lib.wino_probe_launch.restype = ctypes.c_int
        q = lib.wino_probe_queue()
        # 1. correctness, 2 layers, 5 boards
        ws = [(rng.standard_normal((128, 128, 3, 3)) * np.sqrt(2.0 / 1152)).astype(np.float32) for _ in range(2)]
        bs = [(rng.standard_normal(128) * 0.1).astype(np.float32) for _ in range(2)]
        x = bf16_round(torch.relu(torch.randn(5, 64, 128)))
        U = pack_u(ws, q).to(dev)
        bias = torch.from_numpy(np.stack(bs)).to(dev)
        xg = x.to(torch.bfloat16).view(torch.int16).to(dev)
        out = torch.zeros_like(xg)
        run(lib, xg, U, bias, 5, 2, out)
        torch.cuda.synchronize()
        got = out.cpu().view(torch.bfloat16).float()
        ref = reference(x, ws, bs)
        err = (got - ref).abs().max().item()
        scale = ref.abs().max().item()
        # 2. timing, 18 layers, 4096 boards
        L = 18
        ws18 = [ws[i % 2] for i in range(L)]
        U18 = pack_u(ws18, q).to(dev)
        b18 = torch.from_numpy(np.stack([bs[i % 2] for i in range(L)])).to(dev)
        xb = bf16_round(torch.relu(torch.randn(4096, 64, 128))).to(torch.bfloat16).view(torch.int16).to(dev)
        ob = torch.zeros_like(xb)
        t_w = timed(lambda: run(lib, xb, U18, b18, 4096, L, ob))
        t_d = timed(lambda: net(xin))
        t_w2 = timed(lambda: run(lib, xb, U18, b18, 4096, L, ob))
        tw = min(t_w, t_w2)
        flops18 = 2.0 * 64 * 9 * 128 * 128 * 18 * 4096
        print(json.dumps({"lib": Path(path).name, "queue": q, "check_boards": 5, "check_layers": 2,
                          "max_abs_err": round(err, 5), "ref_max_abs": round(scale, 3),
                          "rel_err": round(err / scale, 5),
                          "winograd_18_layers_ms": round(tw, 4), "direct_full_forward_ms": round(t_d, 4),
                          "direct_tower_18_of_19_ms": round(t_d * 18 / 19, 4),
                          "winograd_over_direct_tower": round(tw / (t_d * 18 / 19), 3),
                          "winograd_equiv_TFLOP_s": round(flops18 / (tw * 1e-3) / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()

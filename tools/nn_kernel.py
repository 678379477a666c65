"""Standalone timing of the fused ResNet kernel (csrc/resnet.hip) through
NativeNet's fp32-input forward, for A/Bs of kernel variants and PMC passes
(tools/gpu.sh recipes nn / nnpmc / variants).

Env: ROWS (default 4096), NN_C (128 -> 128x10b, 256 -> 256x20b), NN_BLOCKS
(conv block + residual blocks, default 10 / 20), NN_NET (torch-default
[default], live, frontier, selfplay: bench.py bench_state_dict), NN_REAL=1
(planes of real positions instead of random binary planes), NN_DTYPE
(bf16 / fp16), AB_REF (save the outputs there on the first call, compare bit
for bit on later ones), CHECK_REF=1 (max error of the first 256 rows against
the fp32 restatement oracle/resnet_ref.py; test infrastructure, diagnostics).
Prints one line: ms per launch (median of 5 x 10 launches), TFLOP/s."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))
import torch  # noqa: E402

import othello_mcts as om  # noqa: E402
sys.path.insert(0, str(ROOT))
from bench import bench_state_dict  # noqa: E402
from othello_mcts.synthetic import alphazero_state_dict, calibration_features  # noqa: E402

rows = int(os.environ.get("ROWS", "4096"))
C = int(os.environ.get("NN_C", "128"))
dtype = os.environ.get("NN_DTYPE", "bf16")
R = int(os.environ.get("NN_BLOCKS", "10" if C == 128 else "20")) - 1
kind = os.environ.get("NN_NET", "torch-default")
sd = alphazero_state_dict(1, 17, C, R, C) if kind == "torch-default" else bench_state_dict(kind, 2025, 17, C, R, C)
net = om.NativeNet(sd, device=0, dtype=dtype)
flops = 2.0 * 64 * 9 * C * (17 + 2 * R * C) + 2.0 * (64 * C * 3 + 128 * 65 + 64 * C + C)  # bench.py
if os.environ.get("NN_REAL"):
    x = torch.from_numpy(calibration_features(rows, 8, 7)).cuda()
else:
    x = (torch.rand((rows, 17, 8, 8), generator=torch.Generator().manual_seed(7)) < 0.3).float().cuda()
for _ in range(3):
    net(x)
torch.cuda.synchronize()
ms = []
for _ in range(5):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        net(x)
    b.record()
    torch.cuda.synchronize()
    ms.append(a.elapsed_time(b) / 10)
ms.sort()
t = ms[len(ms) // 2]
out = net(x)
torch.cuda.synchronize()
chk = ""
ref_file = os.environ.get("AB_REF")
if ref_file:  # schedule variants must not change a bit
    if not os.path.exists(ref_file):
        torch.save({k: t_.cpu() for k, t_ in out.items()}, ref_file)
        chk = " [saved reference outputs]"
    else:
        ref = torch.load(ref_file, weights_only=True)
        same = all(torch.equal(ref[k], out[k].cpu()) for k in ref)
        chk = " [outputs bit-identical]" if same else " [OUTPUTS DIFFER]"
if os.environ.get("CHECK_REF"):
    sys.path.insert(0, str(ROOT / "oracle"))
    import resnet_ref  # noqa: E402

    ref = resnet_ref.forward(sd, x[:256])
    chk += (f" [vs fp32: max|dp|={(ref['policy'] - out['policy'][:256]).abs().max().item():.2e}"
            f" max|dv|={(ref['value'] - out['value'][:256]).abs().max().item():.2e}]")
print(f"k_resnet {C}x{R + 1}b {dtype} {kind}{' real' if os.environ.get('NN_REAL') else ''}: {t:.4f} ms/launch  {flops * rows / t / 1e9:.1f} TFLOP/s  (rows={rows}){chk}",
      flush=True)

"""Diagnostic: time the fused ResNet kernel (or an ablation variant selected by
OAMD_RESNET_ABLATE, extension built with OAMD_EXTRA_FLAGS=-DOAMD_ABLATION).
Ablation variants produce wrong outputs; only their timings matter.
Prints one line: variant, ms per launch (median of 5 x 10 launches), TFLOP/s."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))
import torch  # noqa: E402

import othello_mcts as om  # noqa: E402
from othello_mcts.synthetic import alphazero_state_dict  # noqa: E402

rows = int(os.environ.get("ROWS", "8192"))
v = os.environ.get("OAMD_RESNET_ABLATE", "0")
C = int(os.environ.get("NN_C", "128"))  # 128 -> 128x10b, 256 -> 256x20b
R = 9 if C == 128 else 19
sd = alphazero_state_dict(1, 17, C, R, C)
net = om.NativeNet(sd, device=0)
flops = 2.0 * 64 * 9 * C * (17 + 2 * R * C) + 2.0 * (64 * C * 3 + 128 * 65 + 64 * C + C)  # bench.py
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
# schedule variants must not change a bit: compare with the saved reference
out = net(x)
torch.cuda.synchronize()
chk = ""
ref_file = os.environ.get("AB_REF")
if ref_file:
    # variants that change the K order (OAMD_KPERM) have their own reference;
    # every variant is also compared with the first (baseline) reference
    base_file = ref_file
    if "OAMD_KPERM=1" in os.environ.get("AB_FLAGS", ""):
        ref_file = ref_file + ".kperm"
    if not os.path.exists(ref_file):
        torch.save({k: t_.cpu() for k, t_ in out.items()}, ref_file)
        chk = " [saved reference outputs]"
    else:
        ref = torch.load(ref_file, weights_only=True)
        same = all(torch.equal(ref[k], out[k].cpu()) for k in ref)
        chk = " [outputs bit-identical]" if same else " [OUTPUTS DIFFER]"
    if ref_file != base_file and os.path.exists(base_file):
        b = torch.load(base_file, weights_only=True)
        chk += (f" [vs baseline max|dp|={(b['policy'] - out['policy'].cpu()).abs().max().item():.2e}"
                f" max|dv|={(b['value'] - out['value'].cpu()).abs().max().item():.2e}]")
if os.environ.get("CHECK_REF"):  # accuracy vs the fp32 restatement (oracle/resnet_ref.py), first 256 rows
    sys.path.insert(0, str(ROOT / "oracle"))
    import resnet_ref  # noqa: E402
    ref = resnet_ref.forward(sd, x[:256])
    chk += (f" [vs fp32: max|dp|={(ref['policy'] - out['policy'][:256]).abs().max().item():.2e}"
            f" max|dv|={(ref['value'] - out['value'][:256]).abs().max().item():.2e}]")
print(f"variant {v}: {t:.3f} ms/launch  {flops * rows / t / 1e9:.1f} TFLOP/s  (rows={rows}){chk}", flush=True)

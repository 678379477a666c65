"""Diagnostic: where a k_resnet launch spends its time, per workgroup, from the
in-kernel stamps of an OAMD_STAMPS build (OAMD_EXTRA_FLAGS=-DOAMD_STAMPS
python othello-alphazero_amd/build.py --force). One launch of ROWS rows after
warm-up; prints the prologue / tower / heads split, the gap between one
workgroup's exit and the next workgroup's entry on the same CU (dispatch), the
launch's tail (CUs idle while the last workgroups finish) and the tower clock.
"""
import ctypes
import os
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "othello-alphazero_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import othello_mcts as om  # noqa: E402
from othello_mcts.synthetic import alphazero_state_dict  # noqa: E402

rows = int(os.environ.get("ROWS", "8192"))
dtype = os.environ.get("NN_DTYPE", "bf16")
net = om.NativeNet(alphazero_state_dict(1, 17, 128, 9, 128), device=0, dtype=dtype)
x = (torch.rand((rows, 17, 8, 8), device="cuda") < 0.3).float()
for _ in range(20):
    net(x)
torch.cuda.synchronize()
lib = ctypes.CDLL(str(ROOT / "othello-alphazero_amd" / "othello_mcts" / "liboamd.so"))
wgs = rows // 4
STRIDE = 24  # resnet.hip kStampStride
buf = (ctypes.c_uint64 * (wgs * STRIDE))()
assert lib.oamd_debug_read_stamps(buf, ctypes.c_int64(wgs * STRIDE)) == 0, "build with -DOAMD_STAMPS"
s = np.frombuffer(buf, dtype=np.uint64).reshape(wgs, STRIDE).astype(np.int64)
t0, t1, t2, t3, hw, c1, c2, t7, h0, h1, h2, e0, e1, e2 = (s[:, i] for i in range(14))
cu_key = ((hw >> 32) << 8) | ((hw >> 8) & 0xFF)  # XCC id, SE/SH/CU fields of HW_ID
ns = 10.0  # s_memrealtime: 100 MHz
base = t0.min()
span = (t3.max() - base) * ns / 1e3
pro = (t1 - t0) * ns / 1e3
tow = (t2 - t1) * ns / 1e3
hd = (t3 - t2) * ns / 1e3
clk = (c2 - c1) / ((t2 - t1) * ns)  # GHz
per_cu = defaultdict(list)
for i in range(wgs):
    per_cu[int(cu_key[i])].append(i)
gaps, first, last_end = [], [], []
for cu, idx in per_cu.items():
    idx.sort(key=lambda i: t0[i])
    first.append((t0[idx[0]] - base) * ns / 1e3)
    last_end.append((t3[idx[-1]] - base) * ns / 1e3)
    for a, b in zip(idx, idx[1:]):
        gaps.append((t0[b] - t3[a]) * ns / 1e3)
gaps = np.array(gaps)
last_end = np.array(last_end)
busy = (pro + tow + hd).sum()
print(f"rows {rows}: {wgs} workgroups on {len(per_cu)} CUs, launch span {span:.1f} us")
pin = (t7 - t0) * ns / 1e3
print(f"prologue split (median us): entry->inputs staged {np.median(pin):.2f}, stage-0 wait + barrier + first reads {np.median(pro - pin):.2f}")
print(f"heads split (median us): entry {np.median(h0 - t2) * ns / 1e3:.2f}, 1x1 convs (MFMA) "
      f"{np.median(h1 - h0) * ns / 1e3:.2f}, Linear partials {np.median(h2 - h1) * ns / 1e3:.2f}, "
      f"softmax/value + stores {np.median(t3 - h2) * ns / 1e3:.2f}")
print(f"per workgroup (median us): prologue {np.median(pro):.2f}  tower {np.median(tow):.1f}  heads {np.median(hd):.2f}"
      f"  (p90 prologue {np.percentile(pro, 90):.2f}, heads {np.percentile(hd, 90):.2f})")
print(f"same-CU gap exit->next entry: median {np.median(gaps):.2f} us, p90 {np.percentile(gaps, 90):.2f}, "
      f"sum over CUs {gaps.sum() / len(per_cu):.1f} us per CU")
print(f"first entry per CU: median {np.median(first):.2f} us, max {max(first):.2f}; "
      f"tail (span - CU's last exit): median {np.median(span - last_end):.1f} us, max {np.max(span - last_end):.1f}")
print(f"shares of CU time (span x CUs): prologue {pro.sum() / (span * len(per_cu)):.2%}, "
      f"heads {hd.sum() / (span * len(per_cu)):.2%}, tower {tow.sum() / (span * len(per_cu)):.2%}, "
      f"idle {1 - busy / (span * len(per_cu)):.2%}")
if e0.any():
    tc = (c2 - c1).astype(float)
    print(f"epilogues (19 per tower, share of tower cycles, median): first barrier {np.median(e0 / tc):.2%}, "
          f"stores {np.median(e1 / tc):.2%}, second barrier + next layer's first reads {np.median(e2 / tc):.2%}")
print(f"tower clock (s_memtime / s_memrealtime): median {np.median(clk):.3f} GHz")
# all 8 waves' cycle sums (slots 16-22): where a wave's tower time goes
wsum = s[:, 16:23].sum(axis=0).astype(float)
if wsum[6] > 0:
    names = ["step-start lgkmcnt(0) (fragment reads)", "stage-open vmcnt (weight DMA)", "stage barrier",
             "epilogue first barrier", "epilogue stores", "epilogue second barrier + first reads"]
    print("share of the 8 waves' tower cycles: " + ", ".join(f"{n} {wsum[i] / wsum[6]:.2%}" for i, n in enumerate(names))
          + f"; rest (MFMA issue, fragment-read issue, VALU) {1 - wsum[:6].sum() / wsum[6]:.2%}")

"""Tolerance study for a Winograd F(2x2, 3x3) tower: the
tower of a benched net with the kernel's roundings emulated on the CPU —
direct convolution (bf16 / fp16 weights and activations, fp32 accumulation:
reproduces the GPU's measured errors) against F(2x2, 3x3) with bf16 / fp16
transformed inputs V = B^T d B and weights U = G g G^T and fp32 M and
output transform — each against the reference AlphaZeroNet's outputs
(tests/golden/resnet_live.npz). Build container only (CPU):
    python tools/winograd_numerics.py [positions] > profiles/r05/winograd_numerics.json
"""
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
for _p in (ROOT / "tests", ROOT / "othello-alphazero_amd", ROOT / "oracle"):
    sys.path.insert(0, str(_p))
import ref_fixtures as RF  # noqa: E402
import resnet_ref as R  # noqa: E402

dt = torch.bfloat16


def rnd(x):
    return x.to(dt).to(torch.float32)



# F(2x2, 3x3) transforms (Lavin & Gray 2016): Y = A^T [(G g G^T) . (B^T d B)] A
BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float64)
G = torch.tensor([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], dtype=torch.float64)
AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)


def fold(sd, conv, norm):
    """conv + eval BatchNorm folded into weights and a shift (the kernel's packing)."""
    t = {k: torch.as_tensor(sd[k]).double() for k in (conv + ".weight", conv + ".bias", norm + ".weight",
                                                       norm + ".bias", norm + ".running_mean", norm + ".running_var")}
    s = t[norm + ".weight"] / torch.sqrt(t[norm + ".running_var"] + 1e-5)
    shift = t[norm + ".bias"] + (t[conv + ".bias"] - t[norm + ".running_mean"]) * s
    return t[conv + ".weight"] * s[:, None, None, None], shift


def conv_direct(x, w):
    """activations already rounded, weights rounded, exact accumulation"""
    return F.conv2d(x.double(), rnd(w.float()).double(), padding=1)


def conv_wino(x, w):
    """16 tiles of 2x2 outputs per 8x8 board; V and U rounded to the dtype"""
    n = x.shape[0]
    d = F.pad(x.double(), (1, 1, 1, 1)).unfold(2, 4, 2).unfold(3, 4, 2)  # N C ty tx 4 4
    v = rnd(torch.einsum("ai,ncxyij,bj->ncxyab", BT, d, BT).float()).double()
    u = rnd(torch.einsum("ai,ocij,bj->ocab", G, w, G).float()).double()
    m = torch.einsum("ncxyab,ocab->noxyab", v, u)
    y = torch.einsum("pa,noxyab,qb->noxypq", AT, m, AT)  # N O ty tx 2 2
    return y.permute(0, 1, 2, 4, 3, 5).reshape(n, -1, 8, 8)


def forward(sd, x, conv):
    """the tower; activations rounded to the dtype between convs, as in LDS"""
    h = rnd(x.float())
    w, sh = fold(sd, "conv_block.conv", "conv_block.norm")
    h = rnd(F.relu(conv(h, w) + sh[None, :, None, None]).float())
    i = 0
    while f"residual_blocks.{i}.conv1.weight" in sd:
        p = f"residual_blocks.{i}"
        skip = h
        w, sh = fold(sd, p + ".conv1", p + ".norm1")
        h = rnd(F.relu(conv(h, w) + sh[None, :, None, None]).float())
        w, sh = fold(sd, p + ".conv2", p + ".norm2")
        h = rnd(F.relu(conv(h, w) + sh[None, :, None, None] + skip.double()).float())
        i += 1
    return h


def heads(sd, h):
    """fp32 heads (resnet_ref's)"""
    t = {k: torch.as_tensor(v) for k, v in sd.items()}
    pol = F.relu(R._bn(R._conv(h, t, "policy_head.conv", "cpu", 0), t, "policy_head.norm", "cpu"))
    pol = torch.softmax(F.linear(pol.flatten(1), R._t(t, "policy_head.linear.weight", "cpu"),
                                 R._t(t, "policy_head.linear.bias", "cpu")), 1)
    val = F.relu(R._bn(R._conv(h, t, "value_head.conv", "cpu", 0), t, "value_head.norm", "cpu"))
    val = F.relu(F.linear(val.flatten(1), R._t(t, "value_head.linear1.weight", "cpu"),
                          R._t(t, "value_head.linear1.bias", "cpu")))
    val = torch.tanh(F.linear(val, R._t(t, "value_head.linear2.weight", "cpu"),
                              R._t(t, "value_head.linear2.bias", "cpu")).squeeze(1))
    return pol, val


def main():
    global dt
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    out = {"positions": n, "cases": []}
    for name in RF.LIVE_CASES:
        meta, sd, x, g = RF.live_case(name)
        x = torch.from_numpy(x[:n]).float()
        gp, gv = torch.from_numpy(g["policy"][:n]), torch.from_numpy(g["value"][:n])
        for dname, d in (("bf16", torch.bfloat16), ("fp16", torch.float16)):
            dt = d
            for lab, conv in (("direct", conv_direct), ("winograd_f2x2_3x3", conv_wino)):
                p, v = heads(sd, forward(sd, x, conv).float())
                rec = {"net": name, "dtype": dname, "conv": lab,
                       "max_abs_dpolicy": round((p - gp).abs().max().item(), 6),
                       "max_abs_dvalue": round((v - gv).abs().max().item(), 6),
                       "rms_dvalue": round(((v - gv) ** 2).mean().sqrt().item(), 6)}
                out["cases"].append(rec)
                print(json.dumps(rec), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    torch.set_num_threads(8)
    main()

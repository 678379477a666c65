"""ORACLE — TEST INFRASTRUCTURE ONLY.

Plain-PyTorch fp32 restatement of the reference ResNet forward in eval mode
(python/othello_alphazero/neural_net.py):
  ConvBlock      :9-29    conv3x3 + BN + ReLU
  ResidualBlock  :32-65   conv3x3 + BN + ReLU, conv3x3 + BN, + skip, ReLU
  PolicyHead     :68-93   conv1x1(C->2) + BN + ReLU, flatten (c*64+s), Linear, softmax
  ValueHead      :96-128  conv1x1(C->1) + BN + ReLU, Linear, ReLU, Linear, tanh
  AlphaZeroNet   :138-172
It takes the reference state_dict (numpy or torch tensors) and is pinned
against the reference's own outputs in tests/golden/resnet.npz. It is the
fp32 yardstick for the HIP kernels (tolerances in tests/test_gpu_resnet.py).
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

BN_EPS = 1e-5  # torch.nn.BatchNorm2d default


def _t(sd, k, device):
    v = sd[k]
    if not isinstance(v, torch.Tensor):
        v = torch.as_tensor(v)
    return v.to(device=device, dtype=torch.float32)


def _bn(x, sd, p, device):
    return F.batch_norm(
        x,
        _t(sd, p + ".running_mean", device),
        _t(sd, p + ".running_var", device),
        _t(sd, p + ".weight", device),
        _t(sd, p + ".bias", device),
        training=False,
        eps=BN_EPS,
    )


def _conv(x, sd, p, device, pad):
    return F.conv2d(x, _t(sd, p + ".weight", device), _t(sd, p + ".bias", device), padding=pad)


@torch.no_grad()
def forward(sd, x: torch.Tensor) -> dict[str, torch.Tensor]:
    device = x.device
    x = x.to(torch.float32)
    h = F.relu(_bn(_conv(x, sd, "conv_block.conv", device, 1), sd, "conv_block.norm", device))
    i = 0
    while f"residual_blocks.{i}.conv1.weight" in sd:
        p = f"residual_blocks.{i}"
        skip = h
        h = F.relu(_bn(_conv(h, sd, p + ".conv1", device, 1), sd, p + ".norm1", device))
        h = _bn(_conv(h, sd, p + ".conv2", device, 1), sd, p + ".norm2", device)
        h = F.relu(h + skip)
        i += 1
    pol = F.relu(_bn(_conv(h, sd, "policy_head.conv", device, 0), sd, "policy_head.norm", device))
    pol = F.linear(pol.flatten(1), _t(sd, "policy_head.linear.weight", device),
                   _t(sd, "policy_head.linear.bias", device))
    pol = torch.softmax(pol, dim=1)
    val = F.relu(_bn(_conv(h, sd, "value_head.conv", device, 0), sd, "value_head.norm", device))
    val = F.relu(F.linear(val.flatten(1), _t(sd, "value_head.linear1.weight", device),
                          _t(sd, "value_head.linear1.bias", device)))
    val = F.linear(val, _t(sd, "value_head.linear2.weight", device),
                   _t(sd, "value_head.linear2.bias", device))
    val = torch.tanh(val.squeeze(1))
    return {"policy": pol, "value": val}

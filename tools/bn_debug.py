"""Diagnose fused-vs-torch BasicBlock gradient differences under bf16 autocast
(per-branch gradients of one block, identity residual in fp32)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
from torch import nn

import svdformer_pointsea_amd.batchnorm as BN
import svdformer_pointsea_amd.svdformer as S

dev = torch.device("cuda:0")
torch.manual_seed(3)
blk = S.BasicBlock(32, 32, 1, None).to(dev).to(memory_format=torch.channels_last)
with torch.no_grad():
    for m in blk.modules():
        if isinstance(m, nn.BatchNorm2d):
            m.weight.uniform_(0.5, 1.5)
            m.bias.uniform_(-0.2, 0.2)
x = torch.randn(6, 32, 40, 40, device=dev).contiguous(memory_format=torch.channels_last)


def run(enabled):
    BN.ENABLED = enabled
    m = copy.deepcopy(blk)
    xg = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        h = m.conv1(xg)
        h.retain_grad()
        a = BN.bn_act(h, m.bn1, BN.ACT_RELU)
        a.retain_grad()
        c = m.conv2(a)
        c.retain_grad()
        y = BN.bn_act(c, m.bn2, BN.ACT_RELU, residual=xg)
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(1)).to(dev, y.dtype)
    (y.float() * dy.float()).sum().backward()
    return dict(y=y.float(), gx=xg.grad.float(), gh=h.grad.float(), ga=a.grad.float(), gc=c.grad.float())


A, B = run(True), run(False)
for k in A:
    d = (A[k] - B[k]).abs()
    bad = (d > 0.05 + 0.02 * B[k].abs()).float().mean().item()
    print(f"{k}: dtype fused/torch max|d| {d.max().item():.4g} frac bad {bad:.4f}  "
          f"strides {A[k].stride()} / {B[k].stride()}")

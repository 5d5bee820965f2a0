"""libpcops 3x3 conv vs torch (MIOpen, bf16) at the image encoder's full shapes
(96 images: C=16 at 224^2, C=32 at 112^2): relative errors of y, dx, dw and timings.
    python tools/conv_check.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

import svdformer_pointsea_amd.conv as CV

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True
for C, HW in [(16, 224), (32, 112)]:
    g = torch.Generator(device=dev).manual_seed(C)
    x = torch.randn(96, C, HW, HW, device=dev, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(C, C, 3, 3, device=dev, generator=g) / (3 * C ** 0.5)).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(x.shape, device=dev, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    res = {}
    for name in ("pcops", "miopen"):
        xg = x.clone().requires_grad_(True)
        wg = w.clone().requires_grad_(True)
        for it in range(4):
            xg.grad = wg.grad = None
            torch.cuda.synchronize()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            y = CV._Conv3x3.apply(xg, wg) if name == "pcops" else F.conv2d(xg, wg, padding=1)
            e[1].record()
            y.backward(dy)
            e[2].record()
            torch.cuda.synchronize()
        res[name] = (y.float(), xg.grad.float(), wg.grad.float(), e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2]))
        print(f"C={C} {HW}^2 {name}: fwd {res[name][3]:.3f} ms  bwd {res[name][4]:.3f} ms  "
              f"finite y/dx/dw {[bool(torch.isfinite(t).all()) for t in res[name][:3]]}", flush=True)
    for i, k in enumerate(("y", "dx", "dw")):
        a, b = res["pcops"][i], res["miopen"][i]
        print(f"   {k}: rel diff {((a - b).norm() / b.norm()).item():.3e}  max abs {(a - b).abs().max().item():.3e}",
              flush=True)

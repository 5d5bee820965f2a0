"""PCSA apply kernel timing at the SVDFormer / PointSea shapes (channels_last
(B, C, S, K) features, bf16), forward + backward, HIP events per launch.
PCOPS_PCSA_V1=1 selects the block-per-patch kernels (A/B)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from svdformer_pointsea_amd import _lib
from svdformer_pointsea_amd.svdformer import PCSA

tag = "v1" if os.environ.get("PCOPS_PCSA_V1") == "1" else "wave"
for B, C, S, K in [(32, 128, 512, 16), (32, 256, 128, 16), (16, 128, 512, 16)]:
    m = PCSA(C, K).cuda()
    x = torch.randn(B, C, S, K, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    for _ in range(3):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        y.float().sum().backward()
    torch.cuda.synchronize()
    _lib.KernelTimer.enable()
    for _ in range(10):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        y.float().sum().backward()
    torch.cuda.synchronize()
    s = _lib.KernelTimer.summary()
    _lib.KernelTimer.disable()
    mb = B * C * S * K * 2 / 1e6
    f, b = s["pcsa_forward"][1], s["pcsa_backward"][1]
    print(f"[{tag}] B={B} C={C} S={S} K={K}: fwd {f:.3f} ms ({2 * mb / f:.0f} GB/s) | "
          f"bwd {b:.3f} ms ({3 * mb / b:.0f} GB/s)", flush=True)

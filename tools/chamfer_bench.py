"""Chamfer forward at the step's shapes (B=32), HIP-event timed; short enough
to run under rocprofv3 --pmc.  PCOPS_LIB_PATH selects an A/B build of
libpcops; PCOPS_CHAMFER_Q / PCOPS_CHAMFER_SCREEN select the kernel.

    python tools/chamfer_bench.py [iters] [NxM ...]   (default 16384x16384)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svdformer_pointsea_amd.chamfer3D import chamfer_3DDist  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
shapes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[2:]] or [(16384, 16384)]
tag = f"{os.environ.get('PCOPS_LIB_PATH', 'default')} Q={os.environ.get('PCOPS_CHAMFER_Q', 'auto')} " \
      f"screen={os.environ.get('PCOPS_CHAMFER_SCREEN', '1')} cull={os.environ.get('PCOPS_CHAMFER_CULL', '1')} " \
      f"data={os.environ.get('CH_DATA', 'gauss')}"
for N, M in shapes:
    g = torch.Generator(device="cpu").manual_seed(N + M)
    a = (torch.randn(32, N, 3, generator=g) * 0.45).to(dev)
    b = (torch.randn(32, M, 3, generator=g) * 0.45).to(dev)
    if os.environ.get("CH_DATA") == "blob":   # xyz1 collapsed to a tiny blob (a random-init coarse output)
        a = (torch.randn(32, N, 3, generator=g) * 1e-4 + 0.05).to(dev)
        b = (b / b.norm(dim=-1, keepdim=True) * torch.tensor([0.5, 0.3, 0.15], device=dev)).contiguous()
    if os.environ.get("CH_DATA") == "same":   # xyz1: every point the same (a collapsed coarse output)
        a = torch.full((32, N, 3), 0.05, device=dev)
        b = (b / b.norm(dim=-1, keepdim=True) * torch.tensor([0.5, 0.3, 0.15], device=dev)).contiguous()
    if os.environ.get("CH_DATA") == "surface":  # ellipsoid surfaces (completion-like clouds)
        a = (a / a.norm(dim=-1, keepdim=True) * torch.tensor([0.5, 0.3, 0.15], device=dev)).contiguous()
        b = (b / b.norm(dim=-1, keepdim=True) * torch.tensor([0.5, 0.3, 0.15], device=dev)).contiguous()
    for _ in range(3):
        chamfer_3DDist()(a, b)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        chamfer_3DDist()(a, b)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / n
    print(f"{tag}: chamfer 32x{N}x{M} {ms:.4f} ms, {8 * 2 * 32 * N * M / ms / 1e9:.1f} TFLOP/s (8 FLOP/pair)",
          flush=True)

"""Chamfer forward at the loss's 16384 x 16384 shape (B=32), HIP-event timed;
short enough to run under rocprofv3 --pmc.  PCOPS_LIB_PATH selects an A/B
build of libpcops."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svdformer_pointsea_amd.chamfer3D import chamfer_3DDist  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
a = (torch.randn(32, 16384, 3, generator=g) * 0.45).to(dev)
b = (torch.randn(32, 16384, 3, generator=g) * 0.45).to(dev)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
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
print(f"{os.environ.get('PCOPS_LIB_PATH', 'default')}: chamfer 32x16384^2 {ms:.3f} ms, "
      f"{8 * 2 * 32 * 16384 ** 2 / ms / 1e9:.1f} TFLOP/s (8 FLOP/pair)", flush=True)

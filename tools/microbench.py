"""Per-op timing on cuda:0 (HIP events), for development."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svdformer_pointsea_amd.chamfer3D import chamfer_3DDist  # noqa: E402
from svdformer_pointsea_amd.model_utils import _knn  # noqa: E402
from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample  # noqa: E402


def timeit(fn, iters=5, warm=2):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
gt = (torch.randn(32, 16384, 3, generator=g) * 0.45).to(dev)
pr = (torch.randn(32, 16384, 3, generator=g) * 0.45).to(dev)
small = gt[:, :2048].contiguous()
print("fps 32x16384->2048 ms", timeit(lambda: furthest_point_sample(gt, 2048)))
print("fps 32x2048->512 ms", timeit(lambda: furthest_point_sample(small, 512)))
print("fps 32x2048->256 ms", timeit(lambda: furthest_point_sample(small, 256)))
ms = timeit(lambda: chamfer_3DDist()(pr, gt))
print("chamfer 32x16384^2 ms", ms, "Gpairs/s", 2 * 32 * 16384 * 16384 / ms / 1e6)
print("chamfer 32x2048^2 ms", timeit(lambda: chamfer_3DDist()(small, small)))
q = small[:, :512].contiguous()
print("knn3 32x512x2048 k16 ms", timeit(lambda: _knn(q, small, 16)))
print("knn3 self 32x2048 k16 ms", timeit(lambda: _knn(small, small, 16)))
f = torch.randn(32, 512, 64, device=dev)
print("knn64 self 32x512 k8 ms", timeit(lambda: _knn(f, f, 8)))

from svdformer_pointsea_amd.attention import attention_core  # noqa: E402

for (L, Lk, E, H) in [(2048, 2048, 512, 8), (2048, 2048, 1024, 8), (2048, 512, 512, 8), (512, 512, 768, 8),
                      (128, 128, 512, 4)]:
    B = 32
    q = torch.randn(L, B, E, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(Lk, B, E, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(Lk, B, E, device=dev, dtype=torch.bfloat16, requires_grad=True)
    fl = 4.0 * B * L * Lk * E
    ms = timeit(lambda: attention_core(q, k, v, H))
    o = attention_core(q, k, v, H)
    g = torch.randn_like(o)
    msb = timeit(lambda: torch.autograd.grad(o, (q, k, v), g, retain_graph=True))
    print(f"attn bf16 L{L}xLk{Lk} E{E} H{H}: fwd {ms:.3f} ms {fl / ms / 1e9:.1f} TF/s; bwd {msb:.3f} ms "
          f"{2.5 * fl / msb / 1e9:.1f} TF/s")
    qf, kf, vf = q.float().detach(), k.float().detach(), v.float().detach()
    msf = timeit(lambda: attention_core(qf, kf, vf, H), iters=2, warm=1)
    print(f"   fp32 fwd {msf:.3f} ms {fl / msf / 1e9:.1f} TF/s")

"""LayerNorm(+residual) forward/backward kernels vs torch at the block shapes."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from svdformer_pointsea_amd import attention as A


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


for rows, C in [(65536, 1024), (65536, 512), (16384, 768)]:
    norm = torch.nn.LayerNorm(C).cuda()
    a = torch.randn(rows, C, device="cuda", requires_grad=True)
    b = torch.randn(rows, C, device="cuda").bfloat16().requires_grad_(True)
    g32 = torch.randn(rows, C, device="cuda")
    g16 = torch.randn(rows, C, device="cuda").bfloat16()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y32, y16 = A.layer_norm(norm, a, b)
    fwd = timeit(lambda: A._LayerNorm.apply(a, b, norm.weight, norm.bias, norm.eps, True))

    def bwd():
        torch.autograd.backward([y32, y16], [g32, g16], retain_graph=True)
    t_b = timeit(bwd)
    fb = rows * C * (4 + 2 + 4 + 2)
    bb = rows * C * (4 + 2 + 4 + 2 + 4 + 2)
    x = (a.detach() + b.detach().float()).requires_grad_(True)
    yt = torch.nn.functional.layer_norm(x, (C,), norm.weight, norm.bias)
    t_tf = timeit(lambda: torch.nn.functional.layer_norm(x, (C,), norm.weight, norm.bias))
    t_tb = timeit(lambda: torch.autograd.backward([yt], [g32], retain_graph=True))
    print(f"rows={rows} C={C}: fwd {fwd:.3f} ms ({fb / fwd / 1e6:.0f} GB/s)  bwd {t_b:.3f} ms "
          f"({bb / t_b / 1e6:.0f} GB/s) | torch fwd {t_tf:.3f} bwd {t_tb:.3f}", flush=True)

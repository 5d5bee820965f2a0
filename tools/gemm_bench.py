"""bf16 GEMM rates at the attention-block shapes of the PCN step (tokens =
B*L = 65536): forward x @ W^T (+bias), input-grad g @ W, weight-grad
g^T @ x -- hipBLASLt via torch, optionally with the committed TunableOp
selections (argv[1] == 'tuned')."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1 and sys.argv[1] == "tuned":
    from bench import setup_tunableop
    setup_tunableop("use", "svdformer", 0)

dev = torch.device("cuda:0")


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


T = int(os.environ.get('GEMM_T', 65536))
for (cin, cout) in [(512, 1536), (512, 512), (512, 1024), (1024, 512), (1024, 3072), (1024, 1024), (768, 2304)]:
    x = torch.randn(T, cin, device=dev, dtype=torch.bfloat16)
    w = torch.randn(cout, cin, device=dev, dtype=torch.bfloat16)
    b = torch.randn(cout, device=dev, dtype=torch.bfloat16)
    g = torch.randn(T, cout, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * T * cin * cout
    f = timeit(lambda: torch.nn.functional.linear(x, w, b))
    dg = timeit(lambda: g @ w)
    wg = timeit(lambda: g.t() @ x)
    line = (f"{cin}->{cout}: fwd {f*1e3:.0f}us {fl/f/1e9:.0f}TF | dgrad {dg*1e3:.0f}us {fl/dg/1e9:.0f}TF | "
            f"wgrad {wg*1e3:.0f}us {fl/wg/1e9:.0f}TF")
    for S in (4, 8, 16):  # split-K weight gradient: batched partial GEMMs (fp32 out) + one sum
        gb = g.view(S, T // S, cout).transpose(1, 2)
        xb = x.view(S, T // S, cin)
        ws = timeit(lambda: torch.bmm(gb, xb, out_dtype=torch.float32).sum(0).to(torch.bfloat16))
        line += f" | splitK{S} {ws*1e3:.0f}us {fl/ws/1e9:.0f}TF"
    from svdformer_pointsea_amd.attention import _wgrad
    wp = timeit(lambda: _wgrad(g, x, torch.bfloat16))
    line += f" | product _wgrad {wp*1e3:.0f}us {fl/wp/1e9:.0f}TF"
    ref = (g.t().float() @ x.float())
    err = (torch.bmm(g.view(8, T // 8, cout).transpose(1, 2), x.view(8, T // 8, cin), out_dtype=torch.float32).sum(0)
           - ref).abs().max().item()
    print(line + f" | err {err:.2e}", flush=True)

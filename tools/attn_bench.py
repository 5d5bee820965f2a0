"""Attention core timing at the PCN shapes (B=32), forward and backward,
per libpcops launch (HIP events via _lib.KernelTimer).  PCOPS_ATTN_V1=1 in
the environment selects the first-generation kernels for A/B runs; PCOPS_ATTN_FUSED=0
the two-pass backward for head_dim >= 96 ("bwd" = the one-call backward, credited
10*BH*Lq*Lk*D).  ATTN_BENCH_SUMS=1: the step's form -- q / k / v as windows of one packed
(L, B, 3E) source whose gradient feeds a biased Linear, so the backward passes also form the
in_proj bias column sums (the *_colsum kernels)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from svdformer_pointsea_amd import _lib
from svdformer_pointsea_amd.attention import AttentionCore, attention_core

torch.manual_seed(0)
B = 32
shapes = [  # (Lq, Lk, E, H) seen in the PCN step
    (2048, 2048, 512, 8), (2048, 2048, 1024, 8), (2048, 512, 512, 8), (512, 512, 768, 8), (512, 512, 512, 8),
    (128, 128, 512, 4)]
tag = os.environ.get("PCOPS_LIB_PATH", "v1" if os.environ.get("PCOPS_ATTN_V1") == "1" else "v2")
sel = [int(a) for a in sys.argv[1:]]
for si, (Lq, Lk, E, H) in enumerate(shapes):
    if sel and si not in sel:
        continue
    g = torch.randn(Lq, B, E, device="cuda", dtype=torch.bfloat16)
    if os.environ.get("ATTN_BENCH_SUMS") == "1" and Lq == Lk:
        src = torch.randn(Lq, B, 3 * E, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        meta = (H, 1.0 / (E // H) ** 0.5, E, False, (0, 0), (0, E), (0, 2 * E), (True,))
        run = lambda: AttentionCore.apply(meta, src).backward(g)  # noqa: E731
    else:
        q = torch.randn(Lq, B, E, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn(Lk, B, E, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        v = torch.randn(Lk, B, E, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        run = lambda: attention_core(q, k, v, H).backward(g)  # noqa: E731
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    _lib.KernelTimer.enable()
    for _ in range(10):
        run()
    torch.cuda.synchronize()
    summ = _lib.KernelTimer.summary()
    _lib.KernelTimer.disable()
    hd = E // H
    fl = 4.0 * B * H * Lq * Lk * hd
    out = []
    for name, mult in [("attention forward", 1), ("attention bwd dq", 0.5), ("attention bwd dkv", 2.0),
                       ("attention bwd delta", 0), ("attention bwd", 2.5)]:
        if name not in summ:   # delta is fused into the dq launch (bf16)
            continue
        n, mean, tot = summ[name]
        tf = fl * mult / (mean * 1e-3) / 1e12 if mult else 0
        out.append(f"{name.split(' ', 1)[-1]} {mean:.3f}ms {tf:.0f}TF")
    print(f"{tag} Lq={Lq} Lk={Lk} E={E} H={H} hd={hd}: " + " | ".join(out), flush=True)

"""Run-to-run determinism of the attention core: the same bf16 inputs through
forward (+ backward) N times in one process; prints, per shape and tensor,
how many runs differ bitwise from the first and where the differing elements
sit (query rows, batch, head columns)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from svdformer_pointsea_amd.attention import attention_core  # noqa: E402

SHAPES = [(2, 8, 2048, 2048, 512), (2, 8, 2048, 2048, 1024), (2, 8, 512, 512, 768), (2, 4, 130, 129, 128)]
if os.environ.get("DET_SHAPES"):
    SHAPES = [SHAPES[int(i)] for i in os.environ["DET_SHAPES"].split()]
N = int(os.environ.get("DET_RUNS", "6"))
dev = torch.device("cuda", 0)
for B, H, Lq, Lk, E in SHAPES:
    gen = torch.Generator().manual_seed(Lq + E)
    q, k, v = [torch.randn(L, B, E, generator=gen).to(dev, torch.bfloat16) for L in (Lq, Lk, Lk)]
    g = torch.randn(Lq, B, E, generator=gen).to(dev, torch.bfloat16)
    outs = []
    for _ in range(N):
        qs, ks, vs = [t.clone().requires_grad_(True) for t in (q, k, v)]
        o = attention_core(qs, ks, vs, H)
        o.backward(g)
        outs.append((o.detach().clone(), qs.grad.clone(), ks.grad.clone(), vs.grad.clone()))
    torch.cuda.synchronize()
    for ti, name in enumerate(("o", "dq", "dk", "dv")):
        ref = outs[0][ti]
        nd = 0
        for r in range(1, N):
            x = outs[r][ti]
            if not torch.equal(x, ref):
                nd += 1
                if nd == 1:
                    idx = (x != ref).nonzero()
                    rows = idx[:, 0].unique()
                    print(f"  {name} run {r}: {idx.shape[0]} elements differ; rows {rows[:12].tolist()} "
                          f"(of {rows.numel()}), batch {idx[:, 1].unique().tolist()}, cols {idx[:, 2].unique()[:12].tolist()}, "
                          f"max diff {(x.float() - ref.float()).abs().max().item():.3e}")
        print(f"B{B} H{H} Lq{Lq} Lk{Lk} E{E} {name}: {nd} of {N - 1} runs differ", flush=True)

"""fwd2 vs fwd3 outputs: where do they differ (diagnostic)."""
import math
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import torch  # noqa: E402

from svdformer_pointsea_amd.attention import AttentionCore  # noqa: E402

dev = torch.device("cuda", 0)
for (B, H, Lq, Lk, E) in [(2, 8, 2048, 2048, 512), (1, 8, 333, 250, 512)]:
    g = torch.Generator().manual_seed(7)
    q, k, v = [torch.randn(L, B, E, generator=g).to(dev, torch.bfloat16) for L in (Lq, Lk, Lk)]
    meta = (H, 1.0 / math.sqrt(E // H), E, False, (0, 0), (1, 0), (2, 0))
    outs = {}
    for m in ("0", "1", "2"):
        os.environ["PCOPS_FWD3"] = m
        outs[m] = AttentionCore.apply(meta, q, k, v).float()
    for m in ("1", "2"):
        d = (outs[m] - outs["0"]).abs()
        nz = d.nonzero()
        print(f"shape {(B, H, Lq, Lk, E)} mode {m}: {len(nz)} differing of {d.numel()}, max {d.max().item():.3e}, "
              f"rel {(d.max() / outs['0'].abs().max()).item():.3e}", flush=True)
        if len(nz):
            qi = nz[:, 0]
            print("  q mod 64 histogram:", torch.bincount(qi % 64, minlength=64).tolist()[:64], flush=True)
            print("  heads:", torch.bincount(nz[:, 2] // (E // H), minlength=H).tolist(), flush=True)

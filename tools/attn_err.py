"""Measured fp32 error of the attention core (forward and backward) against float64,
per tests/test_gpu_attention.py SHAPES: max |err| and max |ref| for o, dq, dk, dv.
One JSON line per shape (the bound the parity tests assert is set from these)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from test_gpu_attention import SHAPES, _qkv, _ref  # noqa: E402
from svdformer_pointsea_amd.attention import attention_core  # noqa: E402

dev = torch.device("cuda", 0)
for B, H, Lq, Lk, E in SHAPES:
    q, k, v = _qkv(B, H, Lq, Lk, E, dev, seed=1)
    g = torch.randn(Lq, B, E, generator=torch.Generator().manual_seed(5)).to(dev)
    qs, ks, vs = [t.clone().requires_grad_(True) for t in (q, k, v)]
    o = attention_core(qs, ks, vs, H)
    (o * g).sum().backward()
    qd, kd, vd = [t.double().clone().requires_grad_(True) for t in (q, k, v)]
    od = _ref(qd, kd, vd, H)
    (od * g.double()).sum().backward()
    row = {"shape": [B, H, Lq, Lk, E], "hd": E // H}
    for name, a, b in (("o", o, od), ("dq", qs.grad, qd.grad), ("dk", ks.grad, kd.grad), ("dv", vs.grad, vd.grad)):
        row[name] = {"max_abs_err": (a.double() - b.detach()).abs().max().item(), "max_abs_ref": b.abs().max().item()}
    print(json.dumps(row), flush=True)

"""A/B correctness of attention kernel variants selected by environment switches
(read once per process, so each variant runs in its own process):

  PCOPS_DKV3=1 python tools/attn_variant.py dump out_b.pt
  python tools/attn_variant.py dump out_a.pt
  python tools/attn_variant.py cmp out_a.pt out_b.pt

dump: bf16 forward + backward of the attention core at the PCN shapes (B = 2)
and ragged ones; prints each gradient's max |err| against float64 on the same
bf16 inputs and saves o / dq / dk / dv.  cmp: bitwise equality per tensor (and
the max difference where not equal)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

SHAPES = [  # (B, H, Lq, Lk, E)
    (2, 8, 2048, 2048, 1024), (2, 8, 2048, 2048, 512), (2, 8, 2048, 512, 512), (2, 8, 512, 512, 768),
    (3, 2, 200, 333, 256), (1, 4, 77, 130, 256), (2, 2, 1000, 64, 192), (1, 2, 5, 300, 256), (2, 4, 130, 129, 128),
]


def ref(q, k, v, H):
    L, B, E = q.shape
    hd = E // H
    f = lambda t: t.reshape(t.shape[0], B * H, hd).transpose(0, 1)
    s = torch.bmm(f(q), f(k).transpose(1, 2)) / hd ** 0.5
    o = torch.bmm(torch.softmax(s, -1), f(v))
    return o.transpose(0, 1).reshape(L, B, E)


def dump(path):
    from svdformer_pointsea_amd.attention import attention_core
    dev = torch.device("cuda", 0)
    out = {}
    for B, H, Lq, Lk, E in SHAPES:
        gen = torch.Generator().manual_seed(Lq * 7 + Lk + E)
        q, k, v = [torch.randn(L, B, E, generator=gen).to(dev, torch.bfloat16) for L in (Lq, Lk, Lk)]
        g = torch.randn(Lq, B, E, generator=gen).to(dev, torch.bfloat16)
        qs, ks, vs = [t.clone().requires_grad_(True) for t in (q, k, v)]
        o = attention_core(qs, ks, vs, H)
        o.backward(g)
        qd, kd, vd = [t.double().clone().requires_grad_(True) for t in (q, k, v)]
        od = ref(qd, kd, vd, H)
        od.backward(g.double())
        key = f"{B}x{H}x{Lq}x{Lk}x{E}"
        row = {"shape": key}
        for name, a, b in (("o", o, od), ("dq", qs.grad, qd.grad), ("dk", ks.grad, kd.grad), ("dv", vs.grad, vd.grad)):
            row[name] = round((a.double() - b.detach()).abs().max().item() / max(b.abs().max().item(), 1e-30), 6)
            out[key + "/" + name] = a.detach().cpu()
        print(json.dumps(row), flush=True)
    torch.save(out, path)


def cmp(pa, pb):
    a, b = torch.load(pa, weights_only=True), torch.load(pb, weights_only=True)
    bad = 0
    for key in a:
        x, y = a[key], b[key]
        if torch.equal(x, y):
            continue
        bad += 1
        d = (x.float() - y.float()).abs().max().item()
        print(f"DIFF {key}: max |a - b| = {d:.3e} (max |a| {x.float().abs().max().item():.3e})")
    print(f"{len(a) - bad} of {len(a)} tensors bitwise equal")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(1 if cmp(sys.argv[2], sys.argv[3]) else 0)

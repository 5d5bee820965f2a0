"""LayerNorm backward outputs of one libpcops build (PCOPS_LIB_PATH selects an A/B build) over the entry
points and operand configurations the blocks use, saved for a bitwise comparison between builds:

    PCOPS_LIB_PATH=... python tools/ln_ab_cmp.py save out.pt
    python tools/ln_ab_cmp.py cmp a.pt b.pt
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    if sys.argv[1] == "cmp":
        x, y = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
        bad = [k for k in x if not torch.equal(x[k], y[k])]
        print(f"{len(x) - len(bad)} of {len(x)} tensors bitwise equal", *bad)
        sys.exit(1 if bad else 0)
    from svdformer_pointsea_amd import _lib
    from svdformer_pointsea_amd._lib import lib, ptr, stream_of

    dev = torch.device("cuda:0")
    out = {}
    for rows, C in ((65536, 1024), (65536, 512), (16384, 768), (300, 256)):
        for adt, bdt in ((torch.float32, torch.bfloat16), (torch.bfloat16, None), (torch.float32, None)):
            for mode in ("plain", "colsum", "ex_bf16", "ex_gx"):
                g = torch.Generator().manual_seed(rows + C)
                a = torch.randn(rows, C, generator=g).to(dev, adt)
                b = torch.randn(rows, C, generator=g).to(dev, bdt) if bdt is not None else None
                w = (1 + 0.1 * torch.randn(C, generator=g)).to(dev)
                x = a.float() + (b.float() if b is not None else 0)
                mean, rstd = x.mean(1), 1.0 / torch.sqrt(x.var(1, unbiased=False) + 1e-5)
                g32 = torch.randn(rows, C, generator=g).to(dev)
                g16 = torch.randn(rows, C, generator=g).to(dev, torch.bfloat16)
                gb = torch.randn(rows, C, generator=g).to(dev, torch.bfloat16)
                dx32 = torch.empty(rows, C, device=dev)
                dx16 = torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
                dg, db, ds = torch.empty(C, device=dev), torch.empty(C, device=dev), torch.empty(C, device=dev)
                cs = mode != "plain"
                wsb = (lib().pcops_layernorm_bwd_colsum_workspace_bytes(rows, C) if cs
                       else lib().pcops_layernorm_bwd_workspace_bytes(rows, C))
                ws = _lib.Workspace.get(dev, wsb)
                s = stream_of(a)
                adc, bdc = (0 if adt == torch.float32 else 1), (0 if bdt in (None, torch.float32) else 1)
                src = 0 if adt == torch.float32 else 1
                common = (ptr(a), adc, ptr(b), bdc, ptr(w), ptr(mean), ptr(rstd), rows, C, ptr(dx32), ptr(dx16),
                          ptr(dg), ptr(db))
                if mode == "plain":
                    st = lib().pcops_layernorm_bwd(ptr(g32), ptr(g16), *common, ptr(ws), wsb, s)
                elif mode == "colsum":
                    st = lib().pcops_layernorm_bwd_colsum(ptr(g32), ptr(g16), *common, ptr(ds), src, ptr(ws), wsb, s)
                elif mode == "ex_bf16":
                    st = lib().pcops_layernorm_bwd_ex(ptr(gb), 1, C, None, ptr(g16), *common, ptr(ds), src, ptr(ws),
                                                      wsb, s)
                else:
                    st = lib().pcops_layernorm_bwd_ex(ptr(g32), 0, C, ptr(gb), ptr(g16), *common, ptr(ds), src,
                                                      ptr(ws), wsb, s)
                assert st == 0, (mode, st)
                torch.cuda.synchronize()
                key = f"{rows}x{C} {adt} {bdt} {mode}"
                for n, t in (("dx32", dx32), ("dx16", dx16), ("dg", dg), ("db", db)) + ((("ds", ds),) if cs else ()):
                    out[f"{key} {n}"] = t.cpu()
    torch.save(out, sys.argv[2])
    print(len(out), "tensors saved")


if __name__ == "__main__":
    main()

"""Chamfer forward outputs of one libpcops build (PCOPS_LIB_PATH selects an A/B build) on the step's shapes
and data kinds, saved for a bitwise comparison between builds:

    PCOPS_LIB_PATH=... python tools/chamfer_ab_cmp.py save out.pt
    python tools/chamfer_ab_cmp.py cmp a.pt b.pt
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = ((16384, 16384), (2048, 8192), (8192, 8192), (2048, 2048), (512, 2048), (2048, 512), (300, 77))


def clouds(N, M, kind, g):
    a = torch.randn(8, N, 3, generator=g) * 0.45
    b = torch.randn(8, M, 3, generator=g) * 0.45
    if kind == "surface":
        a = a / a.norm(dim=-1, keepdim=True) * torch.tensor([0.5, 0.3, 0.15])
        b = b / b.norm(dim=-1, keepdim=True) * torch.tensor([0.5, 0.3, 0.15])
    if kind == "grid":   # exact ties: integer lattice points
        a = torch.randint(-8, 8, (8, N, 3), generator=g).float() * 0.125
        b = torch.randint(-8, 8, (8, M, 3), generator=g).float() * 0.125
    return a.contiguous(), b.contiguous()


def main():
    if sys.argv[1] == "cmp":
        x, y = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
        bad = [k for k in x if not torch.equal(x[k], y[k])]
        print(f"{len(x) - len(bad)} of {len(x)} tensors bitwise equal", *bad)
        sys.exit(1 if bad else 0)
    from svdformer_pointsea_amd.chamfer3D import chamfer_3DDist

    dev = torch.device("cuda:0")
    ch = chamfer_3DDist()
    out = {}
    for N, M in SHAPES:
        for kind in ("gauss", "surface", "grid"):
            g = torch.Generator().manual_seed(N * 7 + M)
            a, b = clouds(N, M, kind, g)
            d1, d2, i1, i2 = ch(a.to(dev), b.to(dev))
            for n, t in zip(("d1", "d2", "i1", "i2"), (d1, d2, i1, i2)):
                out[f"{N}x{M} {kind} {n}"] = t.cpu()
    torch.save(out, sys.argv[2])
    print(len(out), "tensors saved")


if __name__ == "__main__":
    main()

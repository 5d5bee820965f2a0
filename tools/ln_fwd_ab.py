"""LayerNorm forward of one libpcops build (PCOPS_LIB_PATH selects an A/B build) over the operand configurations
the blocks use: outputs saved for a bitwise comparison between builds, and each configuration timed (HIP events):

    PCOPS_LIB_PATH=... python tools/ln_fwd_ab.py save out.pt
    python tools/ln_fwd_ab.py cmp a.pt b.pt
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
    from svdformer_pointsea_amd._lib import lib, ptr, stream_of

    dev = torch.device("cuda:0")
    out = {}
    for rows, C in ((65536, 512), (65536, 1024), (16384, 768), (16384, 512), (300, 256), (4096, 1024)):
        for adt, bdt in ((torch.float32, torch.bfloat16), (torch.bfloat16, None), (torch.float32, None),
                         (torch.float32, torch.float32)):
            for outs in ("both", "y16"):
                g = torch.Generator().manual_seed(rows + C)
                a = torch.randn(rows, C, generator=g).to(dev, adt)
                b = torch.randn(rows, C, generator=g).to(dev, bdt) if bdt is not None else None
                w = (1 + 0.1 * torch.randn(C, generator=g)).to(dev)
                be = (0.1 * torch.randn(C, generator=g)).to(dev)
                y32 = torch.empty(rows, C, device=dev) if outs == "both" else None
                y16 = torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
                mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
                adc = 0 if adt == torch.float32 else 1
                bdc = -1 if bdt is None else (0 if bdt == torch.float32 else 1)
                s = stream_of(a)

                def run():
                    st = lib().pcops_layernorm_fwd(ptr(a), adc, ptr(b), bdc, ptr(w), ptr(be), 1e-5, rows, C, ptr(y32),
                                                   ptr(y16), ptr(mean), ptr(rstd), s)
                    assert st == 0, st

                for _ in range(3):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                n = 20
                e0.record()
                for _ in range(n):
                    run()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / n
                nbytes = rows * C * (a.element_size() + (b.element_size() if b is not None else 0) + 2
                                     + (4 if y32 is not None else 0))
                key = f"{rows}x{C} {adt} {bdt} {outs}"
                print(f"{key:60s} {ms * 1e3:8.1f} us  {nbytes / ms / 1e9:6.2f} TB/s", flush=True)
                for nm, t in (("y32", y32), ("y16", y16), ("mean", mean), ("rstd", rstd)):
                    if t is not None:
                        out[f"{key} {nm}"] = t.cpu()
    torch.save(out, sys.argv[2])
    print(len(out), "tensors saved")


if __name__ == "__main__":
    main()

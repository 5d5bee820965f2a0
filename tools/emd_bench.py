"""EMD on the clock: pcops_emd_forward / _backward at the reference's TRAIN settings
(eps 0.005, 50 iterations: metrics/EMD/README.md:7) on uniform [0, 1) clouds (the reference's own
harness, emd_module.py:90-106, draws torch.rand), B = 32, n = 2048 and 8192.

    python tools/emd_bench.py out.json
    PCOPS_LIB_PATH=svdformer_pointsea_amd/_lib/count/libpcops.so python tools/emd_bench.py --count out.json

The timing run reports ms per forward (50 auction iterations = 151 launches) and per backward, HIP
events around each, median of 5 after a warm-up.  The --count run (the counting build) adds the bid
pairs the auction evaluates: pairs of UNASSIGNED bidders (the algorithm's work) and lane-pairs the scan
executes (whole 256-bidder blocks scan while any of their bidders is unassigned).  Priced per pair at
the bid loop's VALU cost -- the distance (3 sub, mul, 2 fma), v_sqrt_f32, the reference's double-
precision value ((3.0 - (double)sqrt) - (double)price: 2 cvt + 2 add in f64, 1 cvt back) and the
best / second-best compares -- its VALU roof is pairs x issue cycles / (1024 SIMDs x clock).
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = ((32, 2048), (32, 8192))
EPS, ITERS = 0.005, 50
# issue cycles of one bid-loop pair on one SIMD (MI355X_MICROARCH.md 'vector-instruction ISSUE cost':
# 4 per plain f32 op, 8 per transcendental; f64 add / cvt at the FP64 vector rate, half the f32 rate = 8):
# 3 sub + mul + 2 fma + 2 compare/select chains (~4 ops) = 10 x 4, sqrt 8, 2 cvt_f64 + 2 add_f64 + cvt_f32 = 5 x 8
CYCLES_PER_PAIR = 10 * 4 + 8 + 5 * 8


def main():
    count = "--count" in sys.argv
    out_path = [a for a in sys.argv[1:] if not a.startswith("--")][0]
    from svdformer_pointsea_amd import _lib
    from svdformer_pointsea_amd.emd_module import emdModule

    dev = torch.device("cuda:0")
    emd = emdModule()
    res = {}
    fn = None
    if count:
        fn = _lib.lib().pcops_debug_emd_pair_counts
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 2)()
    for B, n in SHAPES:
        g = torch.Generator(device="cpu").manual_seed(n)
        x1 = torch.rand(B, n, 3, generator=g).to(dev).requires_grad_(True)
        x2 = torch.rand(B, n, 3, generator=g).to(dev)
        key = f"B{B} n{n}"
        if count:
            assert fn(buf) == 0
            emd(x1, x2, EPS, ITERS)
            assert fn(buf) == 0
            res[key] = {"active_pairs": int(buf[0]), "lane_pairs": int(buf[1]),
                        "all_pairs": ITERS * B * n * n}
            print(key, res[key], flush=True)
            continue
        fw, bw = [], []
        for rep in range(6):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            x1.grad = None
            e0.record()
            dist, ass = emd(x1, x2, EPS, ITERS)
            e1.record()
            dist.mean().backward()
            e2.record()
            torch.cuda.synchronize()
            if rep:
                fw.append(e0.elapsed_time(e1))
                bw.append(e1.elapsed_time(e2))
        fw.sort()
        bw.sort()
        d = dist.detach()
        res[key] = {"fwd_ms": round(fw[len(fw) // 2], 4), "bwd_ms": round(bw[len(bw) // 2], 4),
                    "emd": float(d.sqrt().mean()), "unassigned": int((ass < 0).sum()),
                    "distinct_targets": int(sum(ass[b].unique().numel() for b in range(B))) / B}
        print(key, res[key], flush=True)
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()

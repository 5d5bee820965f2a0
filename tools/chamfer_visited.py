"""Pairs the culled Chamfer search really evaluates, per launch shape of the bench's train steps
(price chamfer_3D.forward on visited pairs, not all pairs).

Runs eager train steps of the PCN (B = 32) and the ShapeNet-55 PointSea (B = 16) workloads exactly as
bench.py builds them (random init, synthetic clouds, bf16 autocast, Adam / AdamW) on the COUNTING build
of libpcops (`make -C svdformer_pointsea_amd/csrc count`: -DPCOPS_COUNT_PAIRS, its own .so, selected by
PCOPS_LIB_PATH; the product library has no counters).  Around every chamfer_3D.forward launch it reads
and zeroes the device counters (pcops_debug_pair_counts: pass-1 screen lanes, pass-2 exact rows,
reference scans) and files them under the launch's "NxM" shape.  Steps 0..warm-1 are not counted (the
bench times steps after its warm-up); the rest are averaged.

    PCOPS_LIB_PATH=svdformer_pointsea_amd/_lib/count/libpcops.so python tools/chamfer_visited.py out.json

out.json: {"NxM": {"visited_frac", "pass1_frac", "pass2_frac", "ref_frac", "launches", "B"}} where a
fraction is pairs / (2 B N M), both directions of the launch's all-pairs work.
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_path = sys.argv[1]
    steps, warm = int(os.environ.get("VISITED_STEPS", "6")), int(os.environ.get("VISITED_WARM", "3"))
    if "count" not in os.environ.get("PCOPS_LIB_PATH", ""):
        raise SystemExit("set PCOPS_LIB_PATH to the counting build (svdformer_pointsea_amd/_lib/count/libpcops.so)")
    import bench
    from svdformer_pointsea_amd import _lib, chamfer3D

    L = _lib.lib()
    fn = L.pcops_debug_pair_counts
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 3)()
    acc = {}
    state = {"count": False}
    real_call = chamfer3D.call

    def counting_call(what, f, *args):
        if what != "chamfer_3D.forward":
            return real_call(what, f, *args)
        assert fn(buf) == 0
        r = real_call(what, f, *args)
        assert fn(buf) == 0
        if state["count"]:
            B, N, M = args[2], args[3], args[4]
            a = acc.setdefault(f"{N}x{M}", {"B": B, "launches": 0, "p": [0, 0, 0], "allpairs": 0})
            a["launches"] += 1
            a["allpairs"] += 2 * B * N * M
            for i in range(3):
                a["p"][i] += buf[i]
        return r

    chamfer3D.call = counting_call
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = True
    for name, batch in (("svdformer", 32), ("pointsea", 16)):
        wl = bench.Workload(name)
        torch.manual_seed(0)
        model = wl.Model(wl.cfg).to(dev)
        opt = wl.optimizer(model.parameters())
        partial, gt = wl.synth(batch, 1000, dev)
        rng = torch.cuda.default_generators[0] if name == "pointsea" else None
        for s in range(steps):
            state["count"] = s >= warm
            inp = wl.inputs(partial, gt, rng)
            depth = wl.images(inp)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                pcds = model(inp, depth)
                loss = wl.loss(pcds, inp, gt, wl.gt_pyramid(gt))
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            torch.cuda.synchronize()
            print(f"[visited] {name} step {s} loss {float(loss):.4f}", flush=True)
        del model, opt
        torch.cuda.empty_cache()
    res = {}
    for k, a in sorted(acc.items()):
        p1, p2, p3 = a["p"]
        if p1 + p2 + p3 == 0:
            continue   # an all-pairs launch (the screen kernels count nothing): priced on all pairs
        tot = a["allpairs"]
        res[k] = {"B": a["B"], "launches": a["launches"], "visited_frac": (p1 + p2 + p3) / tot,
                  "pass1_frac": p1 / tot, "pass2_frac": p2 / tot, "ref_frac": p3 / tot}
    json.dump(res, open(out_path, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:>12}  launches {v['launches']:3d}  visited {v['visited_frac']:.4f}  (pass1 {v['pass1_frac']:.4f}, "
              f"pass2 {v['pass2_frac']:.4f}, ref {v['ref_frac']:.4f})")


if __name__ == "__main__":
    main()

"""Which small torch ops run in one eager PCN step: aten ops grouped by input shape
(torch.profiler, record_shapes), filtered by a name regex, with their autograd
parents when they run in backward.
    python tools/op_shapes.py [regex] [rows]"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile

from bench import Workload, setup_tunableop
from svdformer_pointsea_amd.train import FlatParams

pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else r"^aten::(add|add_|copy_|to|_to_copy|sum)$")
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 40
dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = True
setup_tunableop("use", "svdformer", 0)
wl = Workload("svdformer")
torch.manual_seed(0)
model = wl.Model(wl.cfg).to(dev)
fp = FlatParams(model, dev, bf16=True)
partial, gt = wl.synth(wl.batch, 1000, dev)


def step():
    fp.zero_grad()
    fp.refresh()
    gts = wl.gt_pyramid(gt)
    inp = wl.inputs(partial, gt, None)
    depth = wl.images(inp)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        pcds = fp.forward(inp, depth)
        loss = wl.loss(pcds, inp, gt, gts)
    loss.backward()
    fp.collect()


for _ in range(2):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
if os.environ.get("GEMM_TABLE"):
    # device time per (GEMM op, input shapes) with the achieved TFLOP/s
    import math
    rowsk = []
    for k in prof.key_averages(group_by_input_shape=True):
        if not re.match(r"^aten::(mm|addmm|bmm|linear|matmul|_addmm_activation|baddbmm)$", k.key):
            continue
        t = k.device_time_total / 1e3  # ms
        shp = k.input_shapes
        try:
            if k.key in ("aten::mm", "aten::addmm"):
                a, b = (shp[0], shp[1]) if k.key == "aten::mm" else (shp[1], shp[2])
                fl = 2.0 * a[0] * a[1] * b[1]
            elif k.key in ("aten::bmm", "aten::baddbmm"):
                a, b = (shp[0], shp[1]) if k.key == "aten::bmm" else (shp[1], shp[2])
                fl = 2.0 * a[0] * a[1] * a[2] * b[2]
            else:
                fl = float("nan")
        except Exception:
            fl = float("nan")
        rowsk.append((t, k.key, str(shp)[:70], k.count, fl))
    for t, key, shp, n, fl in sorted(rowsk, reverse=True)[:rows]:
        tf = fl * n / (t * 1e-3) / 1e12 if t > 0 and not math.isnan(fl) else float("nan")
        print(f"{t:8.3f} ms {n:4d}x {key:14s} {shp:70s} {tf:7.1f} TFLOP/s")
    sys.exit(0)
# parent of each matching op: the enclosing op / autograd node on the CPU timeline
evs = [e for e in prof.events() if e.device_type.name == "CPU"]
counts = {}
for e in evs:
    if not pat.search(e.name):
        continue
    par = e.cpu_parent
    chain = []
    while par is not None and len(chain) < 3:
        chain.append(par.name)
        par = par.cpu_parent
    key = (e.name, str(e.input_shapes)[:80], " < ".join(chain)[:110])
    counts[key] = counts.get(key, 0) + 1
for (name, shp, chain), n in sorted(counts.items(), key=lambda kv: -kv[1])[:rows]:
    print(f"{n:4d}  {name:18s} {shp:80s} {chain}")

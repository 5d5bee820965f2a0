"""Where the step's torch glue kernels (at::native elementwise / copy / reduce / fill / cat)
come from: one eager PCN (or --model pointsea) train step under torch.profiler with
Python stacks; every glue kernel is charged to its launching aten op and the innermost
frame inside svdformer_pointsea_amd/ (or bench.py).  Prints ms per step per site."""
import argparse
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from bench import Workload, setup_tunableop  # noqa: E402
from svdformer_pointsea_amd import _lib  # noqa: E402
from svdformer_pointsea_amd.train import FlatParams, TrainSchedule  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="svdformer")
ap.add_argument("--rows", type=int, default=45)
args = ap.parse_args()
dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = True
setup_tunableop("use", args.model, 0)
wl = Workload(args.model)
torch.manual_seed(0)
model = wl.Model(wl.cfg).to(dev)
fp = FlatParams(model, dev)
opt = wl.optimizer([fp.master()], fused=True)
partial, gt = wl.synth(wl.batch, 1000, dev)
rng = torch.cuda.default_generators[0] if args.model == "pointsea" else None


def step():
    fp.zero_grad()
    fp.refresh()
    with _lib.fork(dev, lane=1, inputs=(gt,)) as br:
        gts = wl.gt_pyramid(gt)
    inp = wl.inputs(partial, gt, rng)
    depth = wl.images(inp)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = wl.loss(fp.forward(inp, depth), inp, gt, br.join(*gts))
    loss.backward()
    fp.collect()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    step()
    torch.cuda.synchronize()

GLUE = ("at::native", "elementwise", "reduce_kernel", "CatArray", "Fill")


def site(ev):
    """(aten op, innermost package frame) of the CPU op that launched a kernel."""
    op = ev
    while op is not None and not op.name.startswith("aten::"):
        op = op.cpu_parent
    name = op.name if op is not None else "?"
    frame = "?"
    cur = op
    while cur is not None:
        for fr in (cur.stack or []):
            if "svdformer_pointsea_amd" in fr or "bench.py" in fr or "metrics" in fr:
                frame = fr.split("/")[-1]
                break
        if frame != "?":
            break
        if "evaluate_function" in cur.name:   # backward: the autograd node that ran it
            frame = cur.name.split(":")[-1].strip()
            break
        cur = cur.cpu_parent
    return name, frame


cost = defaultdict(lambda: [0, 0.0])
total = 0.0
for ev in prof.events():
    if ev.device_type != torch.autograd.DeviceType.CPU:
        continue
    for k in ev.kernels:
        if not any(g in k.name for g in GLUE):
            continue
        key = site(ev)
        cost[key][0] += 1
        cost[key][1] += k.duration / 1e3
        total += k.duration / 1e3
print(f"glue kernels: {total:.3f} ms in one eager step")
for (op, fr), (n, ms) in sorted(cost.items(), key=lambda kv: -kv[1][1])[:args.rows]:
    print(f"{ms:7.3f} ms {n:4d}x  {op:28s} {fr}")

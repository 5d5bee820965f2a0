"""Per-shape timing of libpcops calls in one eager bench step (HIP events per call,
_lib.KernelTimer): for each call name matching the regex, the distinct scalar
argument tuples (pointers dropped) with launches and mean / total microseconds.

    python tools/call_shapes.py [regex] [--model svdformer|pointsea]
"""
import argparse
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bench import Workload, setup_tunableop
from svdformer_pointsea_amd import _lib
from svdformer_pointsea_amd.train import FlatParams

ap = argparse.ArgumentParser()
ap.add_argument("pattern", nargs="?", default="colsum|sum_rows|gelu")
ap.add_argument("--model", default="svdformer")
args = ap.parse_args()
dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = True
setup_tunableop("use", args.model, 0)
wl = Workload(args.model)
torch.manual_seed(0)
model = wl.Model(wl.cfg).to(dev)
fp = FlatParams(model, dev)
opt = wl.optimizer(model.parameters(), fused=True)
partial, gt = wl.synth(wl.batch, 1000, dev)
rng = torch.cuda.default_generators[0] if args.model == "pointsea" else None


def step():  # bench.py's eager step
    fp.zero_grad()
    fp.refresh()
    with _lib.fork(dev, lane=1) as br:
        gts = wl.gt_pyramid(gt)
    inp = wl.inputs(partial, gt, rng)
    depth = wl.images(inp)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = wl.loss(fp.forward(inp, depth), inp, gt, br.join(*gts))
    loss.backward()
    fp.collect()
    opt.step()


for _ in range(4):
    step()
torch.cuda.synchronize()
_lib.KernelTimer.enable()
step()
torch.cuda.synchronize()
spans = _lib.KernelTimer.spans
_lib.KernelTimer.disable()
pat = re.compile(args.pattern)
for name in sorted(spans):
    if not pat.search(name):
        continue
    groups = defaultdict(list)
    for e0, e1, sc in spans[name]:
        key = tuple(a if not (isinstance(a, int) and abs(a) >= 1 << 32) else "p" for a in sc if a is not None)
        groups[key].append(e0.elapsed_time(e1) * 1e3)
    tot = sum(sum(v) for v in groups.values())
    print(f"== {name}: {sum(len(v) for v in groups.values())} calls, {tot:.1f} us")
    for key, us in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {len(us):3d} x {sum(us) / len(us):8.1f} us = {sum(us):8.1f}  args {key}")

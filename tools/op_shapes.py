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

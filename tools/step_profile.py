"""torch.profiler view of one bench step (eager): per-kernel GPU time grouped
into libpcops / GEMM (hipBLASLt) / conv (MIOpen) / elementwise+reduce / other,
then the top kernels.

    python tools/step_profile.py [--model svdformer|pointsea] [--batch B] [--rows 40]
"""
import argparse
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile

from bench import Workload, setup_tunableop
from svdformer_pointsea_amd import _lib
from svdformer_pointsea_amd.train import FlatParams

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="svdformer")
ap.add_argument("--batch", type=int, default=None)
ap.add_argument("--rows", type=int, default=40)
args = ap.parse_args()
dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = True
setup_tunableop("use", args.model, 0)
wl = Workload(args.model)
B = args.batch or wl.batch
torch.manual_seed(0)
model = wl.Model(wl.cfg).to(dev)
fp = FlatParams(model, dev)
opt = wl.optimizer(model.parameters(), fused=True)
partial, gt = wl.synth(B, 1000, dev)
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
with profile(activities=[ProfilerActivity.CUDA]) as prof:
    step()
    torch.cuda.synchronize()

PCOPS = re.compile(r"attn_|ln_|fps_|chamfer_|knn|gather_points|group_points|transpose_add|depth_|points2|grid2|"
                   r"emd_|three_|ball_")
groups, kern = defaultdict(float), defaultdict(lambda: [0, 0.0])
for e in prof.events():
    if e.device_type != torch.autograd.DeviceType.CUDA:
        continue
    t = e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total
    n = e.name
    if PCOPS.search(n):
        g = "libpcops"
    elif n.startswith("Cijk") or "Custom_Cijk" in n or "gemm" in n.lower() and "igemm" not in n:
        g = "gemm"
    elif "conv" in n.lower() or n.startswith("igemm") or "MIOpen" in n or "batched_transpose" in n:
        g = "conv/bn (MIOpen)"
    elif "elementwise" in n or "reduce_kernel" in n or "Cat" in n or "copy" in n:
        g = "torch elementwise/reduce/copy"
    else:
        g = "other"
    groups[g] += t
    kern[n][0] += 1
    kern[n][1] += t
tot = sum(groups.values())
print(f"step GPU time {tot / 1e3:.2f} ms ({args.model}, B={B})")
for g, t in sorted(groups.items(), key=lambda kv: -kv[1]):
    print(f"  {g:34s} {t / 1e3:8.2f} ms  {100 * t / tot:5.1f}%")
print()
for n, (c, t) in sorted(kern.items(), key=lambda kv: -kv[1][1])[:args.rows]:
    print(f"{t / 1e3:8.3f} ms {c:5d}x  {n[:150]}")

if os.environ.get("SHAPES"):
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof2:
        step()
        torch.cuda.synchronize()
    print(prof2.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=args.rows,
                                                               max_name_column_width=30, max_shapes_column_width=100))

if os.environ.get("OPS"):
    # per-shape totals of selected aten ops (e.g. OPS=aten::copy_,aten::add,aten::sum)
    want = set(os.environ["OPS"].split(","))
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof3:
        step()
        torch.cuda.synchronize()
    rows = []
    for e in prof3.key_averages(group_by_input_shape=True):
        if e.key in want:
            t = getattr(e, "self_device_time_total", 0) or getattr(e, "device_time_total", 0)
            rows.append((t, e.count, e.key, str(e.input_shapes)[:160]))
    for t, c, k, s in sorted(rows, reverse=True)[:args.rows]:
        print(f"{t / 1e3:8.3f} ms {c:4d}x {k:14s} {s}")

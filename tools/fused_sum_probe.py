"""Diagnostic: PCN step gradients with the fused bias sums on vs off, eager
and graph-replayed, from identical weights and inputs.  Prints the loss and
the max |grad difference| per parameter group; flags non-finite values."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bench import Workload, setup_tunableop
from svdformer_pointsea_amd import _lib, attention as A
from svdformer_pointsea_amd.train import FlatParams

dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = False
setup_tunableop("use", "svdformer", 0)
wl = Workload("svdformer")
torch.manual_seed(0)
model = wl.Model(wl.cfg).to(dev)
fp = FlatParams(model, dev)
partial, gt = wl.synth(wl.batch, 1000, dev)
names = list(fp._offset.items())


def step():
    fp.zero_grad()
    fp.refresh()
    with _lib.fork(dev, lane=1) as br:
        gts = wl.gt_pyramid(gt)
    inp = wl.inputs(partial, gt, None)
    depth = wl.images(inp)
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        loss = wl.loss(fp.forward(inp, depth), inp, gt, br.join(*gts))
    loss.backward()
    fp.collect()
    return loss.detach()


def run(fused, graph):
    A._FUSED_BIAS_SUM = fused
    if not graph:
        loss = step()
        torch.cuda.synchronize()
        return loss.item(), fp.grad.clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        out = step()
    outs = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        outs.append((out.item(), fp.grad.clone()))
    return outs


side_hits = []
_orig = A._from_linear


def _spy(t):
    r = _orig(t)
    if r and _lib.on_side_stream():
        side_hits.append(tuple(t.shape))
    return r


A._from_linear = _spy
if os.environ.get("REPS"):   # finiteness over many replays, side-stream fusion on / off
    for side in (False, True):
        A._FUSED_SIDE = side
        side_hits.clear()
        A._FUSED_BIAS_SUM = True
        side_s = torch.cuda.Stream()
        side_s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side_s):
            step()
        torch.cuda.current_stream().wait_stream(side_s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            out = step()
        losses = []
        for _ in range(int(os.environ["REPS"])):
            g.replay()
            torch.cuda.synchronize()
            losses.append(out.item())
        nf = sum(1 for v in losses if v != v or abs(v) == float("inf"))
        print(f"FUSED_SIDE={side}: side-stream fused sums {side_hits[:6]} (n={len(side_hits)}); "
              f"non-finite {nf}/{len(losses)}; losses {losses[:3]}", flush=True)
    sys.exit(0)
ref_loss, ref_g = run(False, False)
print("eager unfused loss", ref_loss, "finite grads", bool(torch.isfinite(ref_g).all()))
for fused, graph in [(True, False), (False, True), (True, True)]:
    res = run(fused, graph)
    res = res if graph else [res]
    for k, (l, gr) in enumerate(res):
        bad = ~torch.isfinite(gr)
        d = (gr - ref_g).abs()
        worst = sorted(((d[o:o + p.numel()].max().item(), n) for n, o in names
                        for p in [dict(model.named_parameters())[n]]), reverse=True)[:4]
        print(f"fused={fused} graph={graph} rep={k}: loss {l:.6f} nonfinite {int(bad.sum())} "
              f"max|dg| {d[torch.isfinite(d)].max().item():.3e} worst {[(f'{v:.2e}', n) for v, n in worst]}")

"""Where the step's torch glue ops come from, by bytes moved: one eager PCN (or --model
pointsea) train step under a TorchDispatchMode that records every aten op outside the
libpcops / GEMM / conv calls (copies, casts, cat, elementwise, reductions, fills) with
its output + input bytes and the innermost Python frame in svdformer_pointsea_amd/ or
bench.py.  Backward ops of torch's own autograd nodes have no Python frame: they are
charged to "<autograd>" plus the op -- or, with --nodes, to the autograd node running when
they are issued (a gradient-accumulation add is issued while its PRODUCER runs) and that
node's forward site (anomaly mode records it; slower, same ops).  Prints GB and calls per
site (complements tools/glue_ops.py, whose profiler stacks come back empty on this torch build)."""
import argparse
import os
import sys
import traceback
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from bench import Workload, setup_tunableop  # noqa: E402
from svdformer_pointsea_amd import _lib  # noqa: E402
from svdformer_pointsea_amd.train import FlatParams  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="svdformer")
ap.add_argument("--rows", type=int, default=60)
ap.add_argument("--nodes", action="store_true", help="attribute backward ops to the running autograd node")
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

SKIP = ("mm", "addmm", "bmm", "baddbmm", "convolution", "cudnn", "miopen", "_scaled_dot", "empty", "view",
        "_unsafe_view", "as_strided", "expand", "permute", "transpose", "t", "unsqueeze", "squeeze", "slice",
        "select", "detach", "alias", "split", "unbind", "reshape", "_reshape_alias", "set_", "lift_fresh",
        "record_stream", "is_nonzero", "_local_scalar_dense", "item", "resize_", "_to_copy_noop")


def nbytes(x):
    if isinstance(x, torch.Tensor):
        return x.numel() * x.element_size()
    if isinstance(x, (list, tuple)):
        return sum(nbytes(y) for y in x)
    return 0


def ours(f):
    return "svdformer_pointsea_amd" in f or f.endswith("bench.py") or "/metrics" in f


def node_site():
    node = torch._C._current_autograd_node()
    if node is None:
        return "<autograd>"
    tb = node.metadata.get("traceback_", []) if hasattr(node, "metadata") else []
    site = "?"
    for entry in (tb if isinstance(tb, list) else [tb]):  # formatted frames, outermost first
        head = entry.strip().splitlines()[0] if entry.strip() else ""
        parts = head.split('"')   # File "<path>", line N, in <fn>
        if head.startswith("File ") and len(parts) >= 3 and ours(parts[1]):
            site = f"{os.path.basename(parts[1])}:{parts[2].split(',')[1].split()[-1]}"
    return f"<{node.name()} @ {site}>"


def frame():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if ours(fr.filename):
            return f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}"
    return node_site() if args.nodes else "<autograd>"


class Rec(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.cost = defaultdict(lambda: [0, 0])

    def __torch_dispatch__(self, func, types, a=(), kw=None):
        out = func(*a, **(kw or {}))
        name = func.overloadpacket.__name__
        if not any(name == s or name.startswith(s + ".") for s in SKIP) and not name.startswith("_foreach"):
            b = nbytes(out) + nbytes(list(a))
            if b:
                c = self.cost[(name, frame())]
                c[0] += 1
                c[1] += b
        return out


def step(rec=None):
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


for _ in range(2):
    step()
torch.cuda.synchronize()
rec = Rec()
if args.nodes:
    torch.autograd.set_detect_anomaly(True, check_nan=False)
with rec:
    step()
torch.cuda.synchronize()
tot = sum(v[1] for v in rec.cost.values())
print(f"glue ops: {tot / 1e9:.3f} GB moved in one eager step, {sum(v[0] for v in rec.cost.values())} ops")
for (op, fr), (n, b) in sorted(rec.cost.items(), key=lambda kv: -kv[1][1])[:args.rows]:
    print(f"{b / 1e6:9.1f} MB {n:4d}x  {op:22s} {fr}")

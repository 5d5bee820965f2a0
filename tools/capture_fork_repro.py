"""Repro of the nested-fork graph-capture segfault, one variant per process.

    python tools/capture_fork_repro.py <variant>

Variants (each captures with torch.cuda.graph in global mode after two eager warm-ups, then
replays once and compares with eager):
  copy_only   lane 3 nested in lane 0, the inner block a torch copy only
  fps_only    the inner block the libpcops FPS (forward only, nothing differentiable)
  full        tests/test_gpu_capture_fork.py's minimal case (forward + backward)
  flat_fps    the FPS fork opened from the ORIGIN stream (sibling of lane 0), joined into lane 0
tools/segv_bt.so prints the native backtrace on SIGSEGV / SIGABRT.  Since the round-5 fix a nested
fork under capture runs inline (base="current", the default here), so copy_only / fps_only / full
no longer reach the runtime's cycle; tools/capture_topology.hip still does, torch-free.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
_BT = ctypes.CDLL(os.path.join(ROOT, "tools", "segv_bt.so"))

import torch  # noqa: E402

from svdformer_pointsea_amd import _lib  # noqa: E402
from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample, gather_operation  # noqa: E402


def body(variant, x, w):
    x_cm = x.transpose(1, 2).contiguous()
    if variant == "flat_fps":
        with _lib.fork(x.device, lane=3, inputs=(x_cm,)) as b3:
            idx = furthest_point_sample(x_cm.transpose(1, 2).float().contiguous(), 256)
        with _lib.fork(x.device, inputs=(x_cm,)) as br:
            f = torch.tanh(torch.einsum("oc,bcn->bon", w, x_cm))
            idx = b3.join(idx)
            g = gather_operation(f.contiguous(), idx)
        g = br.join(g)
        body.extra = (f.detach(), g.detach())
        return g.square().sum(), idx
    with _lib.fork(x.device, inputs=(x_cm,)) as br:
        with _lib.fork(x.device, lane=3, inputs=(x_cm,)) as b3:
            if variant == "copy_only":
                idx = (x_cm.transpose(1, 2).contiguous()[:, :256, 0] * 0).int()
            else:
                idx = furthest_point_sample(x_cm.transpose(1, 2).float().contiguous(), 256)
        f = torch.tanh(torch.einsum("oc,bcn->bon", w, x_cm))
        idx = b3.join(idx)
        g = gather_operation(f.contiguous(), idx)
    g = br.join(g)
    return g.square().sum(), idx


def main():
    variant = sys.argv[1]
    dev = torch.device("cuda:0")
    torch.cuda.init()
    _BT.segv_bt_install()   # after torch and the HIP runtime set up their own handlers
    torch.manual_seed(0)
    x = torch.randn(4, 2048, 3, device=dev)
    w = torch.randn(16, 3, device=dev, requires_grad=variant in ("full", "flat_fps"))

    def run():
        w.grad = None
        body.extra = ()
        loss, idx = body(variant, x, w)
        if w.requires_grad:
            loss.backward()
        return (loss.detach(), idx) + body.extra

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ref = [t.clone() for t in run()]
        run()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    print(f"{variant}: capturing", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = run()
    print(f"{variant}: captured; replaying", flush=True)
    g.replay()
    torch.cuda.synchronize()
    ok = all(torch.equal(a, b) for a, b in zip(out, ref))
    print(f"{variant}: replay equal to eager: {ok}", flush=True)
    for k in range(3):
        g.replay()
        torch.cuda.synchronize()
        print(f"  replay {k}: loss {out[0].item()}", flush=True)
    names = ("loss", "idx", "f", "g")
    for name, a, b in zip(names, out, ref):
        print(f"  {name}: equal {torch.equal(a, b)}; graph {a.flatten()[:6].tolist()} eager {b.flatten()[:6].tolist()}; "
              f"mismatches {(a != b).sum().item()} of {a.numel()}", flush=True)
    # a second eager run: is the eager result itself reproducible?
    with torch.cuda.stream(side):
        again = run()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    print(f"  eager run-to-run equal: {all(torch.equal(a, b) for a, b in zip(again, ref))}", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

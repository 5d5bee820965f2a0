"""Repeat tests/test_gpu_capture_fork.py's minimal nested-fork capture several times per variant in
one process and report, per replay, whether loss / idx / w.grad match eager (no asserts).

    python tools/capture_nested_stress.py [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from svdformer_pointsea_amd import _lib  # noqa: E402
from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample, gather_operation  # noqa: E402


def body(x, w, variant):
    x_cm = x.transpose(1, 2).contiguous()
    if variant.startswith("nofork"):
        if "nofps" in variant:   # indices without the FPS kernel
            idx = (torch.arange(256, device=x.device, dtype=torch.int32) * 7 % 2048).expand(x.shape[0], 256).contiguous()
        else:
            idx = furthest_point_sample(x_cm.transpose(1, 2).float().contiguous(), 256)
        if "mm" in variant:      # the w product as a plain matmul instead of einsum
            f = torch.tanh(torch.matmul(w, x_cm))
        else:
            f = torch.tanh(torch.einsum("oc,bcn->bon", w, x_cm))
        if "nogather" in variant:
            return f[:, :, :256].square().sum(), idx
        return gather_operation(f.contiguous(), idx).square().sum(), idx
    with _lib.fork(x.device, inputs=(x_cm,)) as br:
        if variant == "single":
            idx = furthest_point_sample(x_cm.transpose(1, 2).float().contiguous(), 256)
        else:
            with _lib.fork(x.device, lane=3, inputs=(x_cm,), base=variant) as b3:
                idx = furthest_point_sample(x_cm.transpose(1, 2).float().contiguous(), 256)
        f = torch.tanh(torch.einsum("oc,bcn->bon", w, x_cm))
        if variant != "single":
            idx = b3.join(idx)
        g = gather_operation(f.contiguous(), idx)
    g = br.join(g)
    return g.square().sum(), idx


def trial(variant, seed):
    dev = torch.device("cuda:0")
    torch.manual_seed(seed)
    x = torch.randn(4, 2048, 3, device=dev)
    w = torch.randn(16, 3, device=dev, requires_grad=True)

    def run():
        w.grad = None
        loss, idx = body(x, w, variant)
        loss.backward()
        return loss.detach(), idx, w.grad

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ref = [t.clone() for t in run()]
        run()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        w.grad = None
        loss, idx = body(x, w, variant)
        loss.backward()
    gptr = w.grad.data_ptr()
    res = []
    for _ in range(3):
        if "nopoison" not in variant:
            idx.fill_(-7)
            loss.fill_(float("nan"))
            w.grad.fill_(float("nan"))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        gerr = (w.grad - ref[2]).abs().max().item()
        res.append(f"{int(torch.equal(loss, ref[0]))}{int(torch.equal(idx, ref[1]))}:{gerr:.1e}")
    print(f"{variant:8s} seed {seed}: grad ptr same {gptr == w.grad.data_ptr()}; replays (loss idx : grad err) "
          f"{' '.join(res)}", flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    variants = sys.argv[2].split(",") if len(sys.argv) > 2 else ["nofork", "single", "outer", "current"]
    for variant in variants:
        for seed in range(reps):
            trial(variant, seed)


if __name__ == "__main__":
    main()

"""Per-parameter gradient error of a captured model step (replays 1..3) against eager steps.

    python tools/capture_grad_report.py [pointsea|svdformer] [fp32|bf16]

Prints, per replay, the ten parameters with the largest error relative to their eager run-to-run
spread, and the loss.  Diagnostic for tests/test_gpu_capture_fork.py::test_model_step_capture_replays.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import synth_55, synth_pcn  # noqa: E402
from svdformer_pointsea_amd import pointsea, svdformer  # noqa: E402
from svdformer_pointsea_amd.metrics import get_loss_PM  # noqa: E402
from svdformer_pointsea_amd.render import PCViews, PCViews_Real  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "pointsea"
    amp = len(sys.argv) > 2 and sys.argv[2] == "bf16"
    dev = torch.device("cuda:0")
    torch.manual_seed(1)
    if name == "resnet":   # PointSea's ResEncoder alone (MIOpen convs + libpcops BatchNorm)
        model = pointsea.ResEncoder().to(dev).to(memory_format=torch.channels_last)
        partial, gt = synth_55(2, 6, dev)
        depth = PCViews_Real(TRANS=-pointsea.Config55.NETWORK.view_distance).get_img(partial)
        depth = depth.contiguous(memory_format=torch.channels_last)
        model_call = model
        model = torch.nn.Module()
        model.enc = model_call
        model.forward = lambda p, d: (model_call(d),)   # noqa: E731
        loss_fn = lambda outs: outs[0].float().square().mean()  # noqa: E731
    elif name == "pointsea":
        model = pointsea.Model(pointsea.Config55).to(dev)
        partial, gt = synth_55(2, 6, dev)
        depth = PCViews_Real(TRANS=-pointsea.Config55.NETWORK.view_distance).get_img(partial)
        loss_fn = lambda pcds: get_loss_PM(pcds, partial, gt, sqrt=False)[0]  # noqa: E731
    else:
        model = svdformer.Model(svdformer.PCNConfig).to(dev)
        partial, gt = synth_pcn(2, 6, dev)
        depth = PCViews(TRANS=-0.7, RESOLUTION=224).get_img(partial).unsqueeze(1)
        loss_fn = lambda pcds: svdformer.get_loss(pcds, gt)[0]  # noqa: E731
    named = list(model.named_parameters())

    def step():
        for _, p in named:
            p.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=False):
            pcds = model(partial, depth)
            loss = loss_fn(pcds)
        loss.backward()
        return loss.detach()

    def grads():
        return [None if p.grad is None else p.grad.clone() for _, p in named]

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    eager = []
    with torch.cuda.stream(side):
        for _ in range(3):
            l0 = step()
            eager.append((l0.item(), grads()))
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    spread = [None if a is None else max((a - eager[0][1][i]).abs().max().item(),
                                         (eager[2][1][i] - eager[0][1][i]).abs().max().item())
              for i, a in enumerate(eager[1][1])]
    print(f"{name} {'bf16' if amp else 'fp32'} eager losses {[e[0] for e in eager]}", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loss = step()
    for r in range(3):
        g.replay()
        torch.cuda.synchronize()
        rows = []
        for i, (n, p) in enumerate(named):
            ref = eager[0][1][i]
            if ref is None:
                continue
            err = (p.grad - ref).abs().max().item()
            mx = ref.abs().max().item()
            rows.append((err / (spread[i] + 1e-4 * mx + 1e-12), n, err, spread[i], mx))
        rows.sort(reverse=True)
        print(f"replay {r + 1}: loss {loss.item()}; worst (err / (spread + 1e-4 max)):", flush=True)
        for q, n, err, sp, mx in rows[:10]:
            print(f"   {q:9.2f}  {n}  err {err:.3e} spread {sp:.3e} max {mx:.3e}", flush=True)


if __name__ == "__main__":
    main()

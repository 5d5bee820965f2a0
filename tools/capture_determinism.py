"""Is the PointSea B = 2 forward + loss + backward bitwise reproducible eagerly, and does its
captured graph reproduce it?  Prints the losses of 3 eager steps and 3 replays (outputs poisoned
before each replay), bf16 autocast and fp32, with the local-encoder FPS fork on (base="outer").

    python tools/capture_determinism.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import synth_55  # noqa: E402
from svdformer_pointsea_amd import pointsea  # noqa: E402
from svdformer_pointsea_amd.metrics import get_loss_PM  # noqa: E402
from svdformer_pointsea_amd.render import PCViews_Real  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    pointsea._LOCAL_FPS_FORK = os.environ.get("FORK", "1") == "1"
    for amp in (True, False):
        torch.manual_seed(1)
        model = pointsea.Model(pointsea.Config55).to(dev)
        partial, gt = synth_55(2, 6, dev)
        depth = PCViews_Real(TRANS=-pointsea.Config55.NETWORK.view_distance).get_img(partial)
        params = list(model.parameters())

        def step():
            for p in params:
                p.grad = None
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=False):
                pcds = model(partial, depth)
                loss, _ = get_loss_PM(pcds, partial, gt, sqrt=False)
            loss.backward()
            return [loss.detach()] + [t.detach() for t in pcds]

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        eager = []
        with torch.cuda.stream(side):
            for _ in range(3):
                eager.append([t.clone() for t in step()])
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            outs = step()
        graph = []
        for _ in range(3):
            for t in outs:
                t.fill_(float("nan"))
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            graph.append([t.clone() for t in outs])
        tag = "bf16" if amp else "fp32"
        print(f"{tag} eager losses {[e[0].item() for e in eager]}", flush=True)
        print(f"{tag} graph losses {[e[0].item() for e in graph]}", flush=True)
        for name, runs in (("eager", eager), ("graph", graph)):
            same = [all(torch.equal(a, b) for a, b in zip(r, runs[0])) for r in runs[1:]]
            print(f"{tag} {name} run-to-run bitwise: {same}", flush=True)
        print(f"{tag} graph[0] vs eager[0] bitwise: {all(torch.equal(a, b) for a, b in zip(graph[0], eager[0]))}; "
              f"max |d fine2| {(graph[0][3] - eager[0][3]).abs().max().item():.3e}", flush=True)
        del g


if __name__ == "__main__":
    main()

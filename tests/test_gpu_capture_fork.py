"""HIP-graph capture of nested side-stream forks (`_lib.fork` inside `_lib.fork`).

The bench captures the whole train step into a graph in torch's global capture mode; its
independent branches run on side streams opened by `_lib.fork` (the local encoder on lane 0,
the loss's gt FPS chain on lane 1, the ShapeNet-55 input prefetch on lane 2).  Round 4 put the
PointSea local encoder's FPS on lane 3 INSIDE the lane-0 fork and the bench's capture aborted
(DESIGN.md section 1.2 records the cause).  These tests capture nested forks -- a minimal one
and the PointSea forward + backward at B = 2 -- replay them and compare with eager execution.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _nested(x, w):
    from svdformer_pointsea_amd import _lib
    from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample, gather_operation

    x_cm = x.transpose(1, 2).contiguous()                     # (B, 3, N) on the current stream
    with _lib.fork(x.device, inputs=(x_cm,)) as br:           # lane 0
        with _lib.fork(x.device, lane=3, inputs=(x_cm,)) as b3:   # lane 3 inside lane 0
            idx = furthest_point_sample(x_cm.transpose(1, 2).float().contiguous(), 256)
        f = torch.tanh(torch.einsum("oc,bcn->bon", w, x_cm))     # lane-0 work beside the FPS
        idx = b3.join(idx)
        g = gather_operation(f.contiguous(), idx)
    g = br.join(g)
    return g.square().sum(), idx


def test_nested_fork_capture_minimal(dev):
    """lane 3 nested in lane 0: FPS on the inner stream, a differentiable branch on the outer,
    captured forward + backward, replayed twice: outputs, indices and the weight gradient equal
    to eager."""
    torch.manual_seed(0)
    x = torch.randn(4, 2048, 3, device=dev)
    w = torch.randn(16, 3, device=dev, requires_grad=True)

    def run():
        w.grad = None
        loss, idx = _nested(x, w)
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
        loss, idx = _nested(x, w)
        loss.backward()
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(idx, ref[1])
        assert torch.equal(loss, ref[0])
        torch.testing.assert_close(w.grad, ref[2], rtol=1e-6, atol=0)   # float-atomic gather gradient


def test_pointsea_capture_nested_fork(dev, monkeypatch):
    """The PointSea forward + loss + backward at B = 2 (bf16 autocast, as the bench step) with the
    local encoder's FPS on lane 3 nested in the lane-0 local-encoder fork: captured, replayed, and
    compared with an eager step from the same state -- outputs and loss bitwise (no float
    atomics on the forward path at fixed depth images), gradients within float-atomic order."""
    from bench import synth_55
    from svdformer_pointsea_amd import pointsea
    from svdformer_pointsea_amd.metrics import get_loss_PM
    from svdformer_pointsea_amd.render import PCViews_Real

    monkeypatch.setattr(pointsea, "_LOCAL_FPS_FORK", True)
    torch.manual_seed(1)
    model = pointsea.Model(pointsea.Config55).to(dev)
    partial, gt = synth_55(2, 6, dev)
    depth = PCViews_Real(TRANS=-pointsea.Config55.NETWORK.view_distance).get_img(partial)
    params = [p for p in model.parameters()]

    def step():
        for p in params:
            p.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            pcds = model(partial, depth)
            loss, _ = get_loss_PM(pcds, partial, gt, sqrt=False)
        loss.backward()
        return [loss.detach()] + [t.detach() for t in pcds]

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
        ref = [t.clone() for t in step()]
        ref_g = [None if p.grad is None else p.grad.clone() for p in params]
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        outs = step()
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        for a, b in zip(outs, ref):
            assert torch.equal(a, b)
        for p, r in zip(params, ref_g):
            if r is None:
                assert p.grad is None
            else:
                torch.testing.assert_close(p.grad, r, rtol=1e-2, atol=1e-5)

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


def _nested(x, w, base):
    from svdformer_pointsea_amd import _lib
    from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample, gather_operation

    x_cm = x.transpose(1, 2).contiguous()                     # (B, 3, N) on the current stream
    with _lib.fork(x.device, inputs=(x_cm,)) as br:           # lane 0
        with _lib.fork(x.device, lane=3, inputs=(x_cm,), base=base) as b3:   # lane 3 inside lane 0
            idx = furthest_point_sample(x_cm.transpose(1, 2).float().contiguous(), 256)
        f = torch.tanh(torch.einsum("oc,bcn->bon", w, x_cm))     # lane-0 work beside the FPS
        idx = b3.join(idx)
        g = gather_operation(f.contiguous(), idx)
    g = br.join(g)
    return g.square().sum(), idx


@pytest.mark.parametrize("base", ["outer", "current"])
def test_nested_fork_capture_minimal(dev, base):
    """lane 3 nested in lane 0: FPS on the inner stream, a differentiable branch on the outer,
    captured forward + backward, replayed: outputs, indices and the weight gradient equal to
    eager.  base="outer": the inner fork starts from the origin stream (overlap kept);
    base="current": under capture the inner block runs inline.  The graph's outputs are poisoned
    before every replay, so a missing dependency edge cannot hide behind the previous replay's
    (identical) values."""
    torch.manual_seed(0)
    x = torch.randn(4, 2048, 3, device=dev)
    w = torch.randn(16, 3, device=dev, requires_grad=True)

    def run():
        w.grad = None
        loss, idx = _nested(x, w, base)
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
        loss, idx = _nested(x, w, base)
        loss.backward()
    for _ in range(2):
        idx.fill_(-7)
        loss.fill_(float("nan"))
        w.grad.fill_(float("nan"))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(idx, ref[1])
        assert torch.equal(loss, ref[0])
        torch.testing.assert_close(w.grad, ref[2], rtol=1e-6, atol=0)   # float-atomic gather gradient


def test_pointsea_capture_nested_fork(dev, monkeypatch):
    """The PointSea forward + loss + backward at B = 2 with the local encoder's FPS on lane 3 nested
    in the lane-0 local-encoder fork (base="outer"): captured, replayed with its outputs poisoned,
    and compared with an eager step from the same state.  Not bitwise: the step itself is not
    bitwise reproducible EAGERLY (tools/capture_determinism.py: fp32 eager losses differ in the
    7th digit run to run -- the dense GEMM / conv libraries' reduction order; under bf16 autocast
    such differences flip FPS choices on the predicted clouds and move fine2 points by O(1)).  So
    this runs in fp32, where no index flips occurred, at bars 10x the measured eager spread
    (loss 3e-7 relative, outputs 6e-7): a missing stream dependency (a gather racing its FPS
    measured 4e-3 on the loss) fails it."""
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
        step()   # a second eager step: the eager run-to-run spread of every gradient
        spread = [None if p.grad is None else (p.grad - r).abs().max() for p, r in zip(params, ref_g)]
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        outs = step()
    for _ in range(2):
        for t in outs:
            t.fill_(float("nan"))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(outs[0], ref[0], rtol=3e-6, atol=0)
        for a, b in zip(outs[1:], ref[1:]):
            torch.testing.assert_close(a, b, rtol=0, atol=6e-6)
        for (name, p), r, sp in zip(model.named_parameters(), ref_g, spread):
            if r is None:
                assert p.grad is None
            else:
                # within 4x the eager run-to-run spread of that gradient (MIOpen's conv weight
                # gradients vary by ~1e-3 run to run) plus 1e-4 of its largest magnitude
                err = float((p.grad - r).abs().max())
                assert err <= 4 * float(sp) + 1e-4 * float(r.abs().max()) + 1e-8, (name, err, float(sp))

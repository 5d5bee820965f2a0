"""Eager PCN train steps at the headline shape (B = 32, 2048 -> 16384, bf16
autocast, core/train_pcn.py:101-134) with every fused path on: the bias
column sums handed from the LayerNorm / GELU backward launches to the
Linear backward (attention._attach_sum / _take_sum, blocks of
models/model_utils.py:542-629) and the side-stream branches (the local
encoder, the loss's gt FPS chain: _lib.fork).  Every step's loss must be
finite and equal, within bf16 noise, to the same steps with the fused sums
off (separate colsum launches) from identical weights and inputs."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(dev, fused, steps=3):
    from bench import Workload
    from svdformer_pointsea_amd import _lib
    from svdformer_pointsea_amd import attention as A
    from svdformer_pointsea_amd.train import FlatParams, TrainSchedule

    A._FUSED_BIAS_SUM, A._GELU_SUM = fused, fused
    assert _lib.fork.enabled
    wl = Workload("svdformer")
    torch.manual_seed(0)
    model = wl.Model(wl.cfg).to(dev)
    fp = FlatParams(model, dev, bf16=True)
    opt = wl.optimizer([fp.master()], lr=1e-4, fused=True)
    sched = TrainSchedule(opt, "svdformer")
    partial, gt = wl.synth(32, 1000, dev)
    losses = []
    for _ in range(steps):
        fp.zero_grad()
        fp.refresh()
        with _lib.fork(dev, lane=1, inputs=(gt,)) as br:
            gts = wl.gt_pyramid(gt)
        depth = wl.images(partial)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = wl.loss(fp.forward(partial, depth), partial, gt, br.join(*gts))
        loss.backward()
        fp.collect()
        opt.step()
        sched.batch_end()
        losses.append(loss.detach())
    torch.cuda.synchronize()
    out = [float(v) for v in losses]
    grad_finite = bool(torch.isfinite(fp.grad).all())
    del model, fp, opt
    torch.cuda.empty_cache()
    return out, grad_finite


def test_eager_pcn_steps_fused_sums_finite_and_match_unfused(dev):
    from svdformer_pointsea_amd import attention as A

    saved = (A._FUSED_BIAS_SUM, A._GELU_SUM)
    try:
        fused, gf = _run(dev, True)
        plain, gp = _run(dev, False)
    finally:
        A._FUSED_BIAS_SUM, A._GELU_SUM = saved
    print("fused", fused, "separate", plain)
    assert gf and gp
    assert all(v == v and abs(v) != float("inf") for v in fused + plain)
    # same weights and inputs; the fused sums differ from the separate bf16 colsum by one
    # rounding of the bias gradient, so after Adam steps the losses agree to bf16 noise
    for a, b in zip(fused, plain):
        assert abs(a - b) <= 1e-2 * abs(b), (fused, plain)

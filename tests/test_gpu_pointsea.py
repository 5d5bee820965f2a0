"""End-to-end: the PointSea ShapeNet-55 train step (BASELINE configs[4]) on
libpcops vs the CPU path (oracle/cpu_path.py: C restatement of the point ops
and of the PCViews_Real renderer + torch CPU attention), same weights."""
import copy

import pytest
import torch

from bench import synth_55
from oracle.cpu_path import cpu_ops, real_images
from svdformer_pointsea_amd.metrics import get_loss_PM
from svdformer_pointsea_amd.pointsea import Config55, Model
from svdformer_pointsea_amd.render import PCViews_Real

pytestmark = pytest.mark.gpu


def test_pointsea_forward_matches_cpu_path(dev):
    torch.manual_seed(0)
    cpu = Model(Config55).eval()
    gpu = copy.deepcopy(cpu).cuda().eval()
    partial, gt = synth_55(2, 5, "cpu")
    render = PCViews_Real(TRANS=-Config55.NETWORK.view_distance)
    with torch.no_grad():
        d_gpu = render.get_img(partial.cuda())
        out_gpu = gpu(partial.cuda(), d_gpu)
        loss_gpu, _ = get_loss_PM(out_gpu, partial.cuda(), gt.cuda(), sqrt=False)
        with cpu_ops():
            d_cpu = real_images(render, partial)
            out_cpu = cpu(partial, d_cpu)
            loss_cpu, _ = get_loss_PM(out_cpu, partial, gt, sqrt=False)
    torch.testing.assert_close(d_gpu.cpu(), d_cpu, atol=1e-6, rtol=0)
    for a, b in zip(out_gpu, out_cpu):
        assert a.shape == b.shape
        torch.testing.assert_close(a.cpu(), b, atol=2e-3, rtol=0)
    torch.testing.assert_close(loss_gpu.cpu(), loss_cpu, atol=1e-4, rtol=1e-3)


@pytest.mark.parametrize("amp", [False, True])
def test_pointsea_train_step_runs(dev, amp):
    torch.manual_seed(1)
    model = Model(Config55).cuda()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=5e-4)
    partial, gt = synth_55(2, 6, "cuda")
    render = PCViews_Real(TRANS=-Config55.NETWORK.view_distance)
    losses = []
    for _ in range(3):
        depth = render.get_img(partial)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            pcds = model(partial, depth)
            loss, _ = get_loss_PM(pcds, partial, gt, sqrt=False)
        assert [p.shape for p in pcds] == [(2, 256, 3), (2, 2048, 3), (2, 8192, 3)]
        opt.zero_grad(set_to_none=True)
        loss.backward()
        for n, p in model.named_parameters():
            if ".sa_module_" in n and ".bn." in n:
                assert p.grad is None, n
                continue
            assert p.grad is not None and torch.isfinite(p.grad).all(), n
        opt.step()
        losses.append(loss.item())
    assert all(torch.isfinite(torch.tensor(losses)))


def test_seprate_point_cloud_matches_per_sample_loop(dev):
    """Batched zero-padded FPS == the reference's per-sample ragged FPS calls
    (utils/helpers.py:79-119), same crop sizes and centres."""
    import torch.nn.functional as F

    from svdformer_pointsea_amd.data import seprate_point_cloud
    from svdformer_pointsea_amd.model_utils import fps_subsample

    _, gt = synth_55(4, 11, dev)
    n = gt.shape[1]
    crop = [n // 4, 3 * n // 4]
    g = torch.Generator(device=dev).manual_seed(5)
    inp, cr = seprate_point_cloud(gt, n, crop, generator=g)
    g2 = torch.Generator(device=dev).manual_seed(5)
    num_crop = torch.randint(crop[0], crop[1] + 1, (4,), device=dev, generator=g2)
    center = F.normalize(torch.randn(4, 1, 3, device=dev, generator=g2), p=2, dim=-1)
    for b in range(4):
        pts = gt[b:b + 1]
        d = torch.norm(center[b:b + 1].unsqueeze(2) - pts.unsqueeze(1), p=2, dim=-1)
        idx = torch.argsort(d, dim=-1, descending=False)[0, 0]
        k = int(num_crop[b])
        ref_in = fps_subsample(pts[0, idx[k:]].unsqueeze(0).contiguous(), 2048)
        ref_cr = fps_subsample(pts[0, idx[:k]].unsqueeze(0).contiguous(), 2048)
        assert torch.equal(inp[b:b + 1], ref_in)
        assert torch.equal(cr[b:b + 1], ref_cr)


def test_seprate_point_cloud_without_crop_same_input(dev):
    """want_crop=False (the train loop's `partial, _ = ...`, core/train_55.py:150)
    skips the crop part's FPS and returns the same input cloud, bitwise: FPS draws
    no random numbers, so the generator stream is unchanged."""
    from svdformer_pointsea_amd.data import seprate_point_cloud

    _, gt = synth_55(4, 12, dev)
    n = gt.shape[1]
    crop = [n // 4, 3 * n // 4]
    a, ca = seprate_point_cloud(gt, n, crop, generator=torch.Generator(device=dev).manual_seed(7))
    b, cb = seprate_point_cloud(gt, n, crop, generator=torch.Generator(device=dev).manual_seed(7), want_crop=False)
    assert ca is not None and cb is None
    assert torch.equal(a, b)
    for k in (n // 2,):   # fixed crop size: the gather path
        a, _ = seprate_point_cloud(gt, n, k, generator=torch.Generator(device=dev).manual_seed(8))
        b, cb = seprate_point_cloud(gt, n, k, generator=torch.Generator(device=dev).manual_seed(8), want_crop=False)
        assert cb is None and torch.equal(a, b)


def test_pointsea_glue_fusions_match_unfused(dev, monkeypatch):
    """The PointSea SDG glue fusions (path-selection blend in one launch emitting the bf16 conv_ps
    operand; the selection concatenation from bf16 parts) against the plain torch expressions, one
    bf16-autocast forward + backward of the model: outputs bitwise.  The broadcast f_g_current part's
    gradient is summed over a differently laid-out tensor (fp32 reduction order), and a last-bit fp32
    change can flip a later bf16 rounding, so gradients are held to 1e-3 relative L2 per parameter."""
    import svdformer_pointsea_amd.attention as A
    import svdformer_pointsea_amd.pointsea as PS

    torch.manual_seed(2)
    model = Model(Config55).cuda()
    partial, gt = synth_55(2, 7, "cuda")
    render = PCViews_Real(TRANS=-Config55.NETWORK.view_distance)
    depth = render.get_img(partial)

    def run(fused):
        monkeypatch.setattr(A, "_PCOPS_BLEND", fused)
        monkeypatch.setattr(PS, "_CAT16", fused)
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            pcds = model(partial, depth)
            loss, _ = get_loss_PM(pcds, partial, gt, sqrt=False)
        loss.backward()
        return [p.detach().clone() for p in pcds], {n: p.grad.clone() for n, p in model.named_parameters()
                                                     if p.grad is not None}

    # the first call of a conv shape may run a different MIOpen algorithm than later calls (the
    # image encoder's output moved in bf16 between two otherwise identical first passes): warm up
    # once and pin deterministic algorithms, so the comparison sees only the fusions
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    monkeypatch.setattr(torch.backends.cudnn, "benchmark", False)
    run(False)
    (out_a, g_a), (out_b, g_b) = run(True), run(False)
    for x, y in zip(out_a, out_b):
        assert torch.equal(x, y)
    assert g_a.keys() == g_b.keys()
    for n in g_a:
        err = (g_a[n].float() - g_b[n].float()).norm().item()
        assert err <= 1e-3 * g_b[n].float().norm().item() + 1e-8, (n, err)


@pytest.mark.parametrize("which", ["pointsea", "svdformer"])
def test_shared_partial_fps_model_bitwise(dev, monkeypatch, which):
    """The models' one shared FPS of the partial cloud (svdformer.shared_partial_fps: the local
    encoder's local_points FPS, whose first 512 indices are the first SA module's FPS) against the
    two separate FPS calls of the reference (SVDFormer.py:177 / PointSea.py:241 and
    model_utils.py:341): a bf16-autocast forward, outputs bitwise equal -- the indices are the same,
    so is everything computed from them."""
    import svdformer_pointsea_amd.svdformer as SV

    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    monkeypatch.setattr(torch.backends.cudnn, "benchmark", False)
    torch.manual_seed(3)
    if which == "pointsea":
        model = Model(Config55).cuda().eval()
        partial, _ = synth_55(2, 9, "cuda")
        depth = PCViews_Real(TRANS=-Config55.NETWORK.view_distance).get_img(partial)
    else:
        from bench import synth_pcn
        from svdformer_pointsea_amd.render import PCViews
        model = SV.Model(SV.PCNConfig).cuda().eval()
        partial, _ = synth_pcn(2, 9, "cuda")
        depth = PCViews(TRANS=-0.7, RESOLUTION=224).get_img(partial).unsqueeze(1)

    def run(share):
        monkeypatch.setattr(SV, "_FPS_SHARE", share)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            return [p.clone() for p in model(partial, depth)]

    run(True)   # first-call algorithm choices out of the way
    a, b = run(True), run(False)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_seprate_point_cloud_counts_bitwise(dev, monkeypatch):
    """The crop FPS with per-cloud valid counts (pcops_furthest_point_sampling_counts, rows past the
    count skipped) returns the input cloud of the plain zero-padded FPS bitwise, crop part included,
    for random and for fixed crop sizes."""
    import svdformer_pointsea_amd.data as D

    _, gt = synth_55(4, 13, dev)
    n = gt.shape[1]
    for crop in ([n // 4, 3 * n // 4], n // 2, n // 4):
        out = []
        for cnt in (True, False):
            monkeypatch.setattr(D, "_FPS_COUNTS", cnt)
            out.append(D.seprate_point_cloud(gt, n, crop, generator=torch.Generator(device=dev).manual_seed(9)))
        (a, ca), (b, cb) = out
        assert torch.equal(a, b) and torch.equal(ca, cb), crop


@pytest.mark.parametrize("shape,dtype,kind", [((6, 64, 112, 112), torch.bfloat16, "relu"),
                                              ((3, 16, 9, 14), torch.float32, "ties"),
                                              ((2, 24, 15, 8), torch.bfloat16, "nan"),
                                              ((4, 8, 1, 5), torch.float32, "relu")])
def test_stem_maxpool_matches_torch_bitwise(dev, shape, dtype, kind):
    """The ResEncoder stem's nn.MaxPool2d(3, 2, 1) on libpcops (pcops_maxpool3s2_fwd / _bwd) against
    torch's own NHWC kernels: output and input gradient bitwise equal -- ties (the first maximum
    wins), overlapping windows (an element winning several windows sums their gradients in torch's
    order), NaN inputs, odd and single-row images."""
    from torch import nn

    from svdformer_pointsea_amd import pointsea as PS

    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(shape, generator=g)
    if kind == "relu":
        x = x.clamp_min(0)
    elif kind == "ties":
        x = torch.round(x * 2) / 2      # many exact ties inside windows
    else:
        x[:, :, ::3, ::4] = float("nan")
    x = x.to(dev, dtype).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(shape[0], shape[1], (shape[2] + 1) // 2, (shape[3] + 1) // 2, generator=g)
    gy = gy.to(dev, dtype).contiguous(memory_format=torch.channels_last)
    pool = nn.MaxPool2d(3, 2, 1)
    out = []
    for fn in (lambda t: pool(t), lambda t: PS.maxpool3s2(pool, t)):
        xx = x.clone().requires_grad_(True)
        y = fn(xx)
        y.backward(gy)
        out.append((y.detach(), xx.grad))
    torch.testing.assert_close(out[1][0], out[0][0], rtol=0, atol=0, equal_nan=True)
    torch.testing.assert_close(out[1][1], out[0][1], rtol=0, atol=0, equal_nan=True)

"""End-to-end: the SVDFormer PCN train step on libpcops vs the CPU path.

The CPU side is the same model class driven by oracle/cpu_path.py (the C
restatement of the point ops + torch CPU attention), i.e. the reference's
model code on CPU stand-ins.  Weights are copied, so any difference comes
from the hot-path ops and dense-layer rounding (hipBLASLt/MIOpen vs CPU).
"""
import copy

import pytest
import torch

from bench import synth_pcn
from oracle.cpu_path import cpu_ops, depth_images
from svdformer_pointsea_amd.render import PCViews
from svdformer_pointsea_amd.svdformer import Model, PCNConfig, get_loss

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def models():
    torch.manual_seed(0)
    cpu = Model(PCNConfig).eval()
    gpu = copy.deepcopy(cpu).cuda().eval()
    return cpu, gpu


def test_forward_matches_cpu_path(dev, models):
    cpu, gpu = models
    partial, gt = synth_pcn(2, 7, "cpu")
    render = PCViews(TRANS=-0.7, RESOLUTION=224)
    with torch.no_grad():
        d_gpu = render.get_img(partial.cuda()).unsqueeze(1)
        out_gpu = gpu(partial.cuda(), d_gpu)
        loss_gpu, parts_gpu = get_loss(out_gpu, gt.cuda())
        with cpu_ops():
            d_cpu = depth_images(render, partial).unsqueeze(1)
            out_cpu = cpu(partial, d_cpu)
            loss_cpu, parts_cpu = get_loss(out_cpu, gt)
    # same pixels; values equal up to float-atomic summation order (as test_pcviews_*)
    assert torch.equal(d_gpu.cpu() != 0, d_cpu != 0)
    torch.testing.assert_close(d_gpu.cpu(), d_cpu, rtol=1e-6, atol=1e-7)
    for a, b in zip(out_gpu, out_cpu):
        assert a.shape == b.shape
        # dense layers round differently on the GPU; outputs are O(0.5)
        torch.testing.assert_close(a.cpu(), b, atol=2e-3, rtol=0)
    torch.testing.assert_close(loss_gpu.cpu(), loss_cpu, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("amp", [False, True])
def test_train_step_runs(dev, amp):
    torch.manual_seed(1)
    model = Model(PCNConfig).cuda()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    partial, gt = synth_pcn(2, 8, "cuda")
    render = PCViews(TRANS=-0.7, RESOLUTION=224)
    losses = []
    for _ in range(3):
        depth = render.get_img(partial).unsqueeze(1)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            pcds = model(partial, depth)
            loss, _ = get_loss(pcds, gt)
        assert [p.shape for p in pcds] == [(2, 256, 3), (2, 2048, 3), (2, 16384, 3)]
        opt.zero_grad(set_to_none=True)
        loss.backward()
        for n, p in model.named_parameters():
            if ".sa_module_" in n and ".bn." in n:
                # Conv2d(if_bn=False) still owns an unused BatchNorm (model_utils.py:27-43)
                assert p.grad is None, n
                continue
            assert p.grad is not None and torch.isfinite(p.grad).all(), n
        opt.step()
        losses.append(loss.item())
    assert all(torch.isfinite(torch.tensor(losses)))

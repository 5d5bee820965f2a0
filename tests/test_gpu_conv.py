"""pcops_conv3x3_fwd / _wgrad (csrc/conv.hip) against float64 torch.nn.functional.conv2d
on the same bf16-valued inputs: forward, input gradient (the flipped-weight forward)
and weight gradient, at the image encoder's channel counts and at ragged H / W
(partial 4 x 64 tiles, images narrower than one tile); then a BasicBlock with the
libpcops convs against the same block on MIOpen, both measured against float64.

Tolerances: outputs are bf16 roundings of fp32 sums -> rel 2^-8 of the value plus
an atol of 2^-8 * the typical magnitude; the fp32 weight gradient 1e-4 of its norm."""
import copy

import pytest
import torch
import torch.nn.functional as F
from torch import nn

import svdformer_pointsea_amd.batchnorm as BN
import svdformer_pointsea_amd.conv as CV
import svdformer_pointsea_amd.svdformer as S

pytestmark = pytest.mark.gpu

# the last two have more 4 x 64 tiles than the weight gradient has blocks (1024 / 768):
# every block loops over several tiles with the next-tile prefetch
SHAPES = [(2, 16, 40, 70), (3, 32, 17, 129), (1, 16, 5, 3), (2, 32, 64, 64), (1, 16, 224, 224),
          (32, 16, 128, 128), (64, 32, 64, 64)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("wfmt", ["oihw_f32", "ohwi_bf16"])
def test_conv3x3_vs_float64(dev, shape, wfmt):
    N, C, H, W = shape
    g = torch.Generator().manual_seed(N * 1000 + C + H + W)
    x = torch.randn(shape, generator=g).to(torch.bfloat16)
    w = (torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5))
    dy = torch.randn(shape, generator=g).to(torch.bfloat16)
    if wfmt == "ohwi_bf16":
        w = w.to(torch.bfloat16)
    xg = x.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wg = w.to(dev)
    if wfmt == "ohwi_bf16":
        wg = wg.contiguous(memory_format=torch.channels_last)
    wg.requires_grad_(True)
    y = CV._Conv3x3.apply(xg, wg)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    y.backward(dy.to(dev).contiguous(memory_format=torch.channels_last))
    assert wg.grad.dtype == wg.dtype and wg.grad.stride() == wg.stride()

    x64 = x.double().requires_grad_(True)
    w64 = w.to(torch.bfloat16).double().requires_grad_(True)   # the kernel's operands are bf16 (as autocast's)
    y64 = F.conv2d(x64, w64, padding=1)
    y64.backward(dy.double())
    mag = y64.abs().mean().item()
    torch.testing.assert_close(y.double().cpu(), y64.detach(), atol=2 ** -8 * mag, rtol=2 ** -8)
    gmag = x64.grad.abs().mean().item()
    torch.testing.assert_close(xg.grad.double().cpu(), x64.grad, atol=2 ** -8 * gmag, rtol=2 ** -8)
    gw = wg.grad.double().cpu()
    if wfmt == "oihw_f32":
        err = (gw - w64.grad).norm() / w64.grad.norm()
        assert err < 1e-5, err
    else:
        torch.testing.assert_close(gw, w64.grad, atol=2 ** -8 * w64.grad.abs().mean().item(), rtol=2 ** -8)


def test_conv3x3_eligibility(dev):
    conv = nn.Conv2d(16, 16, 3, padding=1, bias=False).to(dev)
    x = torch.randn(2, 16, 8, 8, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert CV.eligible(x, conv)
    assert not CV.eligible(x.float(), conv)                                          # fp32 input: MIOpen
    assert not CV.eligible(x.contiguous(), conv)                                     # NCHW memory
    assert not CV.eligible(x, nn.Conv2d(16, 16, 3, stride=2, padding=1, bias=False).to(dev))
    assert not CV.eligible(x, nn.Conv2d(16, 16, 3, padding=1, bias=True).to(dev))
    x64 = torch.randn(2, 64, 8, 8, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert not CV.eligible(x64, nn.Conv2d(64, 64, 3, padding=1, bias=False).to(dev))


def _run_block(blk, x, conv_on, monkeypatch):
    monkeypatch.setattr(CV, "ENABLED", conv_on)
    m = copy.deepcopy(blk)
    xg = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(xg)
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(1)).to(y.device, y.dtype)
    (y.float() * dy.float()).sum().backward()
    return y.float(), xg.grad.float(), {n: p.grad.float() for n, p in m.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("C,HW", [(16, 56), (32, 28)])
def test_basic_block_conv_vs_miopen(dev, monkeypatch, C, HW):
    torch.manual_seed(C)
    blk = S.BasicBlock(C, C, 1, None).to(dev).to(memory_format=torch.channels_last)
    with torch.no_grad():
        for m in blk.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    x = torch.randn(4, C, HW, HW, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ya, gxa, ga = _run_block(blk, x, True, monkeypatch)
    yb, gxb, gb = _run_block(blk, x, False, monkeypatch)
    # float64 block (torch's modules on the CPU)
    blk64 = copy.deepcopy(blk).double().cpu()
    x64 = x.detach().double().cpu().requires_grad_(True)
    monkeypatch.setattr(BN, "ENABLED", False)
    y64 = blk64(x64)
    dy = torch.randn(y64.shape, generator=torch.Generator().manual_seed(1)).to(torch.bfloat16).double()
    (y64 * dy).sum().backward()
    g64 = {n: p.grad for n, p in blk64.named_parameters() if p.grad is not None}

    def rel(a, ref):
        return ((a.double().cpu() - ref).norm() / ref.norm()).item()

    assert ga.keys() == gb.keys()
    for name, a, b, r in [("y", ya, yb, y64.detach()), ("dx", gxa, gxb, x64.grad)] + \
            [(k, ga[k], gb[k], g64[k]) for k in ga]:
        ea, eb = rel(a, r), rel(b, r)
        # parameter gradients are sums over the batch with cancellation (a bias gradient is
        # sum(dy * mask)): ReLU flips on either path move them by a few %, so a looser margin
        slack = (1.25, 2e-3) if name in ("y", "dx") else (1.5, 2e-2)
        assert ea <= slack[0] * eb + slack[1], f"{name}: libpcops conv rel err {ea:.3g} vs MIOpen {eb:.3g}"


@pytest.mark.parametrize("shape", [(3, 1, 224, 224), (2, 1, 37, 70)])
@pytest.mark.parametrize("wdt", [torch.float32, torch.bfloat16])
def test_stem_conv_vs_float64(dev, shape, wdt):
    """The 1 -> 16 stem: x rounded to bf16 and bf16 weights (autocast's operands), fp32 sums."""
    g = torch.Generator().manual_seed(shape[2])
    x = torch.rand(shape, generator=g) * 2.0
    w = (torch.randn(16, 1, 3, 3, generator=g) / 3).to(wdt)
    dy = torch.randn(shape[0], 16, shape[2], shape[3], generator=g).to(torch.bfloat16)
    wg = w.to(dev).requires_grad_(True)
    y = CV._Conv3x3C1.apply(x.to(dev), wg)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    y.backward(dy.to(dev).contiguous(memory_format=torch.channels_last))
    assert wg.grad.dtype == wdt
    x64 = x.to(torch.bfloat16).double()
    w64 = w.to(torch.bfloat16).double().requires_grad_(True)
    y64 = F.conv2d(x64, w64, padding=1)
    y64.backward(dy.double())
    torch.testing.assert_close(y.double().cpu(), y64.detach(), atol=2 ** -8 * y64.abs().mean().item(), rtol=2 ** -8)
    gw = wg.grad.double().cpu()
    if wdt == torch.float32:
        assert ((gw - w64.grad).norm() / w64.grad.norm()) < 1e-5
    else:
        torch.testing.assert_close(gw, w64.grad, atol=2 ** -8 * w64.grad.abs().mean().item(), rtol=2 ** -8)


def test_stem_eligibility(dev):
    conv = nn.Conv2d(1, 16, 3, padding=1, bias=False).to(dev)
    x = torch.rand(2, 1, 16, 16, device=dev)
    assert not CV.stem_eligible(x, conv)          # needs bf16 autocast (torch would compute in fp32)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert CV.stem_eligible(x, conv)
        assert not CV.stem_eligible(x, nn.Conv2d(1, 16, 3, padding=1, bias=True).to(dev))
        y = CV.conv3x3(x, conv)
    assert y.dtype == torch.bfloat16

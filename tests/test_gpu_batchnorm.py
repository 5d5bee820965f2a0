"""pcops_batchnorm_fwd / _bwd (csrc/batchnorm.hip) against a float64 restatement
of torch.nn.BatchNorm2d (training: biased batch variance, running stats with
the unbiased one; eval: running stats) followed by the residual add and
ReLU / LeakyReLU, on the same channels_last inputs -- and, through the model
code, against torch's own modules (MIOpen) for a ResNet BasicBlock and an
EdgeConv under bf16 autocast.

Tolerances: fp32 outputs / input gradients 2e-5 abs+rel of float64;
bf16 outputs within one bf16 rounding of the float64 value (rel 2^-8);
dgamma / dbeta (fp32 sums over bf16 inputs) 1e-4 rel of float64."""
import copy

import pytest
import torch
from torch import nn

import svdformer_pointsea_amd.batchnorm as BN
import svdformer_pointsea_amd.svdformer as S

pytestmark = pytest.mark.gpu


def _ref(x, res, w, b, rm, rv, training, mom, eps, act, slope, round16=False):
    """float64 BatchNorm2d (+res) (+act); returns y and the updated running stats.
    round16: the BN output is rounded to bf16 before the residual add (torch's bf16
    BatchNorm output as stored; straight-through for the gradient)."""
    xd = x.double()
    C = x.shape[1]
    if training:
        mean = xd.mean(dim=(0, 2, 3))
        var = xd.var(dim=(0, 2, 3), unbiased=False)
        n = x.numel() // C
        rm2 = (1 - mom) * rm.double() + mom * mean
        rv2 = (1 - mom) * rv.double() + mom * var * n / (n - 1)
    else:
        mean, var = rm.double(), rv.double()
        rm2, rv2 = rm.double(), rv.double()
    y = (xd - mean.view(1, C, 1, 1)) / torch.sqrt(var.view(1, C, 1, 1) + eps) * w.double().view(1, C, 1, 1) \
        + b.double().view(1, C, 1, 1)
    if res is not None:
        if round16:
            y = y + (y.to(torch.bfloat16).double() - y).detach()
        y = y + res.double()
    _ref.pre = y.detach()
    if act == BN.ACT_RELU:
        y = torch.relu(y)
    elif act == BN.ACT_LEAKY:
        y = torch.where(y > 0, y, y * slope)
    return y, rm2, rv2


CASES = [  # (N, C, H, W)
    (4, 16, 32, 32),
    (2, 32, 24, 40),
    (3, 64, 12, 12),
    (2, 128, 7, 9),
    (2, 512, 7, 7),
    (5, 24, 10, 10),   # C/8 = 3: odd vector count per row
]


@pytest.mark.parametrize("shape", CASES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act,res", [(BN.ACT_NONE, False), (BN.ACT_RELU, False), (BN.ACT_RELU, True),
                                     (BN.ACT_LEAKY, False)])
def test_bn_act_train_vs_float64(dev, shape, dtype, act, res):
    g = torch.Generator().manual_seed(hash((shape, act, res)) % 1000)
    N, C, H, W = shape
    x = (torch.randn(shape, generator=g) * 1.7 + 0.8).to(dev, dtype).contiguous(memory_format=torch.channels_last)
    r = (torch.randn(shape, generator=g).to(dev, dtype).contiguous(memory_format=torch.channels_last)
         if res else None)
    bn = nn.BatchNorm2d(C).to(dev)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g) * 0.1)
        bn.running_mean.copy_(torch.randn(C, generator=g))
        bn.running_var.copy_(torch.rand(C, generator=g) + 0.5)
    rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
    xg = x.clone().requires_grad_(True)
    rg = r.clone().requires_grad_(True) if res else None
    y = BN.bn_act(xg, bn, act, 0.2, rg)
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    assert int(bn.num_batches_tracked) == 1
    dy = torch.randn(shape, generator=g).to(dev, dtype).contiguous(memory_format=torch.channels_last)
    y.backward(dy)

    xr = x.double().requires_grad_(True)
    rr = r.double().requires_grad_(True) if res else None
    wr = bn.weight.detach().double().requires_grad_(True)
    br = bn.bias.detach().double().requires_grad_(True)
    yr, rm2, rv2 = _ref(xr, rr, wr, br, rm0, rv0, True, 0.1, 1e-5, act, 0.2, round16=dtype == torch.bfloat16)
    yr.backward(dy.double())
    # elementwise gradient checks skip pre-activations within 1e-4 of the kink, where
    # fp32 vs float64 rounding may pick the other side of the activation
    sel = _ref.pre.abs() > 1e-4 if act != BN.ACT_NONE else torch.ones_like(_ref.pre, dtype=torch.bool)

    if dtype == torch.float32:
        torch.testing.assert_close(y.double(), yr.detach(), atol=2e-5, rtol=2e-5)
        torch.testing.assert_close(xg.grad.double()[sel], xr.grad[sel], atol=2e-5, rtol=2e-5)
        if res:
            torch.testing.assert_close(rg.grad.double()[sel], rr.grad[sel], atol=0, rtol=0)
    else:
        torch.testing.assert_close(y.double(), yr.detach(), atol=1e-2, rtol=2 ** -8)
        torch.testing.assert_close(xg.grad.double()[sel], xr.grad[sel], atol=2e-2, rtol=2 ** -7)
        if res:
            torch.testing.assert_close(rg.grad.double()[sel], rr.grad[sel], atol=0, rtol=2 ** -8)
    torch.testing.assert_close(bn.running_mean.double(), rm2, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(bn.running_var.double(), rv2, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(bn.weight.grad.double(), wr.grad, atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(bn.bias.grad.double(), br.grad, atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_act_eval_vs_float64(dev, dtype):
    g = torch.Generator().manual_seed(5)
    shape = (3, 64, 14, 14)
    x = torch.randn(shape, generator=g).to(dev, dtype).contiguous(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(64).to(dev).eval()
    with torch.no_grad():
        bn.weight.copy_(torch.rand(64, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(64, generator=g))
        bn.running_mean.copy_(torch.randn(64, generator=g))
        bn.running_var.copy_(torch.rand(64, generator=g) + 0.5)
    xg = x.clone().requires_grad_(True)
    y = BN.bn_act(xg, bn, BN.ACT_RELU)
    assert int(bn.num_batches_tracked) == 0
    dy = torch.randn(shape, generator=g).to(dev, dtype).contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    xr = x.double().requires_grad_(True)
    yr, _, _ = _ref(xr, None, bn.weight.detach(), bn.bias.detach(), bn.running_mean, bn.running_var, False, 0.1, 1e-5,
                    BN.ACT_RELU, 0.0)
    yr.backward(dy.double())
    sel = _ref.pre.abs() > 1e-4
    tol = dict(atol=2e-5, rtol=2e-5) if dtype == torch.float32 else dict(atol=1e-2, rtol=2 ** -7)
    torch.testing.assert_close(y.double(), yr.detach(), **tol)
    torch.testing.assert_close(xg.grad.double()[sel], xr.grad[sel], **tol)


def test_bn_rows_large_shifted(dev):
    """A (96, 16, 224, 224) activation (the SVFNet layer-1 shape) with a large mean:
    the shifted per-chunk sums keep the variance accurate (no E[x^2] - E[x]^2 cancellation)."""
    g = torch.Generator(device=dev).manual_seed(7)
    x = (torch.randn((96, 16, 224, 224), generator=g, device=dev) * 0.05 + 30.0).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(16).to(dev)
    y = BN.bn_act(x, bn, BN.ACT_NONE)
    xd = x.double()
    mean = xd.mean(dim=(0, 2, 3))
    var = xd.var(dim=(0, 2, 3), unbiased=False)
    ref = (xd - mean.view(1, -1, 1, 1)) / torch.sqrt(var.view(1, -1, 1, 1) + 1e-5)
    torch.testing.assert_close(y.double(), ref, atol=2e-2, rtol=2 ** -7)
    n = x.numel() // 16
    torch.testing.assert_close(bn.running_var.double(), 0.9 + 0.1 * var * n / (n - 1), atol=1e-7, rtol=1e-5)


def _block_grads(mod, x, enabled, monkeypatch, amp):
    monkeypatch.setattr(BN, "ENABLED", enabled)
    m = copy.deepcopy(mod)
    xg = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        y = m(xg)
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(1)).to(y.device, y.dtype)
    (y.float() * dy.float()).sum().backward()
    grads = {n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None}
    bufs = {n: b.float().clone() for n, b in m.named_buffers()}
    return y.float(), xg.grad.float(), grads, bufs


@pytest.mark.parametrize("amp", [False, True])
@pytest.mark.parametrize("down", [False, True])
def test_basic_block_fused_vs_torch(dev, monkeypatch, amp, down):
    torch.manual_seed(3)
    cin, cout, stride = (16, 32, 2) if down else (32, 32, 1)
    ds = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride, bias=False), nn.BatchNorm2d(cout)) if down else None
    blk = S.BasicBlock(cin, cout, stride, ds).to(dev).to(memory_format=torch.channels_last)
    with torch.no_grad():
        for m in blk.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    # under autocast the block input is the previous block's bf16 output (as in SVFNet / ResEncoder)
    x = torch.randn(6, cin, 40, 40, device=dev, dtype=torch.bfloat16 if amp else torch.float32)
    x = x.contiguous(memory_format=torch.channels_last)
    ya, gxa, ga, ba = _block_grads(blk, x, True, monkeypatch, amp)
    yb, gxb, gb, bb = _block_grads(blk, x, False, monkeypatch, amp)
    assert ga.keys() == gb.keys()
    if not amp:
        tol = dict(atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(ya, yb, **tol)
        torch.testing.assert_close(gxa, gxb, **tol)
        for k in ga:
            torch.testing.assert_close(ga[k], gb[k], atol=1e-3, rtol=2e-4)
        for k in ba:
            torch.testing.assert_close(ba[k], bb[k], atol=1e-5, rtol=1e-5)
    else:
        # bf16: MIOpen's bf16 BatchNorm and this one round differently (its statistics are not
        # exact), and one ReLU flipped by a bf16 ulp moves a gradient element by a full dy that
        # the next conv spreads -- so both are measured against the float64 block, and the
        # fused path must be at least as accurate as torch's
        blk64 = copy.deepcopy(blk).double().cpu()
        x64 = x.detach().double().cpu().requires_grad_(True)
        monkeypatch.setattr(BN, "ENABLED", False)
        y64 = blk64(x64)
        dy = torch.randn(y64.shape, generator=torch.Generator().manual_seed(1)).to(torch.bfloat16).double()
        (y64 * dy).sum().backward()
        g64 = {n: p.grad for n, p in blk64.named_parameters() if p.grad is not None}

        def rel(a, ref):
            return ((a.double().cpu() - ref).norm() / ref.norm()).item()

        for name, a, b, r in [("y", ya, yb, y64.detach()), ("dx", gxa, gxb, x64.grad)] + \
                [(k, ga[k], gb[k], g64[k]) for k in ga]:
            ea, eb = rel(a, r), rel(b, r)
            # parameter gradients are sums over the batch with cancellation (a bias gradient is
            # sum(dy * mask)): ReLU flips on either path move them by a few %, so a looser margin
            slack = (1.25, 2e-3) if name in ("y", "dx") else (1.5, 2e-2)
            assert ea <= slack[0] * eb + slack[1], f"{name}: fused rel err {ea:.3g} vs torch {eb:.3g}"
        for k in ba:
            torch.testing.assert_close(ba[k], bb[k], atol=1e-3, rtol=1e-3)


def test_edgeconv_fused_vs_torch(dev, monkeypatch):
    torch.manual_seed(4)
    ec = S.EdgeConv(3, 64, 16).to(dev).to(memory_format=torch.channels_last)
    x = (torch.rand(2, 3, 512, device=dev) - 0.5)
    ya, gxa, ga, ba = _block_grads(ec, x, True, monkeypatch, False)
    yb, gxb, gb, bb = _block_grads(ec, x, False, monkeypatch, False)
    torch.testing.assert_close(ya, yb, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(gxa, gxb, atol=1e-4, rtol=1e-4)
    for k in ga:
        torch.testing.assert_close(ga[k], gb[k], atol=1e-3, rtol=1e-3)
    for k in ba:
        torch.testing.assert_close(ba[k], bb[k], atol=1e-5, rtol=1e-5)


def _bn_run(dev, shape, dtype, act, res, seed):
    g = torch.Generator().manual_seed(seed)
    N, C, H, W = shape
    x = (torch.randn(shape, generator=g) * 1.7 + 0.8).to(dev, dtype).contiguous(memory_format=torch.channels_last)
    r = (torch.randn(shape, generator=g).to(dev, dtype).contiguous(memory_format=torch.channels_last)
         if res else None)
    dy = torch.randn(shape, generator=g).to(dev, dtype).contiguous(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(C).to(dev)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g) * 0.1)
        bn.running_mean.copy_(torch.randn(C, generator=g))
        bn.running_var.copy_(torch.rand(C, generator=g) + 0.5)
    xg = x.clone().requires_grad_(True)
    rg = r.clone().requires_grad_(True) if res else None
    y = BN.bn_act(xg, bn, act, 0.2, rg)
    y.backward(dy)
    out = [y, xg.grad, bn.weight.grad, bn.bias.grad, bn.running_mean, bn.running_var, bn.num_batches_tracked]
    return out + ([rg.grad] if res else [])


@pytest.mark.parametrize("shape", [(4, 16, 32, 32), (3, 64, 12, 12), (2, 128, 7, 9), (8, 64, 56, 56),
                                   (2, 256, 7, 7), (5, 24, 10, 10)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_fused_final_bitwise(dev, monkeypatch, shape, dtype):
    """The final step folded into the statistics pass (the last block of each channel strip to
    finish combines the partial rows, PCOPS_BN_FUSED_FINAL, round 5) gives bitwise the outputs,
    gradients and running statistics of the separate bn_final launch: the same partial rows
    summed in the same order."""
    for act, res in ((BN.ACT_RELU, True), (BN.ACT_LEAKY, False), (BN.ACT_NONE, False)):
        seed = hash((shape, act, res)) % 1000
        monkeypatch.setenv("PCOPS_BN_FUSED_FINAL", "0")
        a = _bn_run(dev, shape, dtype, act, res, seed)
        monkeypatch.setenv("PCOPS_BN_FUSED_FINAL", "1")
        b = _bn_run(dev, shape, dtype, act, res, seed)
        for i, (u, v) in enumerate(zip(a, b)):
            assert torch.equal(u, v), (act, res, i)


def test_bn_fused_final_graph_replays(dev):
    """Captured once and replayed: each replay's fused launches find their arrival counters back
    at zero (the last block resets them), so every replay equals the eager result."""
    shape = (8, 64, 28, 28)
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(shape, generator=g) + 0.3).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(shape, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(64).to(dev)
    xg = x.clone().requires_grad_(True)

    def step():
        xg.grad = None
        bn.weight.grad = bn.bias.grad = None
        y = BN.bn_act(xg, bn, BN.ACT_RELU, 0.0, None)
        y.backward(dy)
        return y.detach()

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        y0 = step().clone()
        ref = [y0, xg.grad.clone(), bn.weight.grad.clone(), bn.bias.grad.clone()]
        step()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        y = step()
    for _ in range(4):
        graph.replay()
        torch.cuda.synchronize()
        got = [y, xg.grad, bn.weight.grad, bn.bias.grad]
        for u, v in zip(ref, got):
            assert torch.equal(u, v)


@pytest.mark.parametrize("C,HW", [(16, 56), (32, 28), (16, 224)])
def test_basic_block_skip_fused_bitwise(dev, monkeypatch, C, HW):
    """A stride-1 BasicBlock's input gradient with the identity's share summed inside conv1's dgrad
    launch (conv._Conv3x3Skip -> pcops_conv3x3_fwd_res) against autograd's separate bf16 add: the
    output, the input gradient and every parameter gradient bitwise equal, bf16 autocast."""
    import svdformer_pointsea_amd.conv as CV

    torch.manual_seed(C + HW)
    blk = S.BasicBlock(C, C).to(dev).to(memory_format=torch.channels_last)
    with torch.no_grad():
        for m in blk.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    x = torch.randn(4, C, HW, HW, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(4, C, HW, HW, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def run(fused):
        monkeypatch.setattr(CV, "SKIP_FUSED", fused)
        m = copy.deepcopy(blk)
        xg = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(xg)
        y.backward(dy)
        return [y.detach(), xg.grad] + [p.grad for p in m.parameters()]

    a, b = run(False), run(True)
    for i, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u, v), i
